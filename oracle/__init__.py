"""TEST INFRASTRUCTURE ONLY — the CPU/fp32 parity oracle for the tair_amd hot path.

This package is a plain-PyTorch fp32 restatement of the reference's ControlLDM denoising path
(yinnhao/TAIR @ 2025-08-08).  It is the *checker*, never the thing measured or shipped:
only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import it.
The product path (``tair_amd``) never imports anything from here and fails loudly when its
HIP extension is missing.

Pinning status: the reference's Python could not be imported or run in
this container (environment denial recorded in SURVEY.md §8c), the reference ships no tests,
golden vectors or offline weights.  The oracle is therefore pinned only by analytic
known-answer tests (respaced timesteps, schedule tables, zero-terminal-SNR identities) and by the
reference's own parameter counts / state-dict layout; its layer numerics are **parity unpinned**
against the reference beyond those checks.
"""
