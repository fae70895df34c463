#!/usr/bin/env python
"""Per-launch cost of small runtime kernels when chained in a hipGraph (no profiler): LayerNorm,
GroupNorm apply and a small split-K GEMM at the B=1 16x16-level shapes, vs torch's tiny add."""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from tair_amd import _lib  # noqa: E402


def timed_graph(fn, n, s):
    with torch.cuda.stream(s):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        for _ in range(n):
            fn()
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / 5 / n * 1000


def main():
    L = _lib.lib()
    dev = "cuda"
    s = torch.cuda.Stream()
    sp = lambda: ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)  # noqa: E731
    n = 200
    x = torch.zeros(64, device=dev)
    print(f"torch add_ (1 block): {timed_graph(lambda: x.add_(1.0), n, s):.2f} us", flush=True)
    for T, C in ((256, 1280), (4096, 320)):
        a = torch.randn(T, C, device=dev).to(torch.bfloat16)
        y = torch.empty_like(a)
        gmm = torch.ones(C, device=dev)
        b = torch.zeros(C, device=dev)
        us = timed_graph(lambda: L.tair_k_layernorm(a.data_ptr(), T, C, gmm.data_ptr(), b.data_ptr(), 1e-5,
                                                    y.data_ptr(), sp()), n, s)
        print(f"layernorm T={T} C={C}: {us:.2f} us", flush=True)
        ss = torch.randn(C * 2, device=dev)
        ws = torch.zeros(32 * 64 * 2, device=dev)
        tk = torch.zeros(32, device=dev, dtype=torch.int32)
        us = timed_graph(lambda: L.tair_k_groupnorm_ex(a.data_ptr(), C, 1, T, C, 32, 1e-5, gmm.data_ptr(),
                                                       b.data_ptr(), 1, y.data_ptr(), C, ss.data_ptr(),
                                                       ws.data_ptr(), tk.data_ptr(), sp()), n, s)
        print(f"groupnorm (stats+apply, 2 launches) HW={T} C={C}: {us:.2f} us", flush=True)
    for M, N, K, sp_ in ((256, 1280, 1280, 0), (256, 1280, 1280, 1), (4096, 320, 320, 0), (1024, 640, 640, 1)):
        A = torch.randn(M, K, device=dev).to(torch.bfloat16)
        W = torch.randn(N, K, device=dev).to(torch.bfloat16)
        out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        part = torch.empty(8 << 20, device=dev)
        d = _lib.GemmDesc()
        d.M, d.N, d.K, d.amode, d.A, d.lda, d.Wt, d.ldw, d.out, d.ldo, d.alpha = \
            M, N, K, 0, A.data_ptr(), K, W.data_ptr(), K, out.data_ptr(), N, 1.0
        d.partial, d.partial_cap, d.force_splits = part.data_ptr(), part.numel(), sp_
        us = timed_graph(lambda: L.tair_k_gemm(ctypes.byref(d), sp()), n, s)
        print(f"gemm {M}x{N}x{K} splits={'heur' if not sp_ else sp_}: {us:.2f} us "
              f"({2 * M * N * K / us / 1e6:.1f} TFLOP/s)", flush=True)


if __name__ == "__main__":
    main()
