#!/usr/bin/env python
"""Time the attention kernel over the network's attention shapes (B=1 by default) for every
(qsets, splits) plan and print the best per shape next to the heuristic's choice."""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from tair_amd import _lib  # noqa: E402

# (Sq, heads, Skv) of the SD-2.1 UNet / ControlNet transformers at a 64x64 latent
SHAPES = [(4096, 5, 4096), (1024, 10, 1024), (256, 20, 256), (64, 20, 64),
          (4096, 5, 77), (1024, 10, 77), (256, 20, 77), (64, 20, 77)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    L = _lib.lib()
    dev = "cuda"
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    ws = torch.empty(64 << 20, device=dev, dtype=torch.uint8)
    B = a.batch
    for Sq, Hh, Skv in SHAPES:
        C = Hh * 64
        q = torch.randn(B * Sq, C, device=dev).to(torch.bfloat16)
        k = torch.randn(B * Skv, C, device=dev).to(torch.bfloat16)
        v = torch.randn(B * Skv, C, device=dev).to(torch.bfloat16)
        o = torch.empty(B * Sq, C, device=dev, dtype=torch.bfloat16)
        flops = 4.0 * B * Sq * Skv * C

        def run(qs, sp):
            return L.tair_k_attention_ex(q.data_ptr(), C, k.data_ptr(), C, v.data_ptr(), C, o.data_ptr(), C, B, Hh,
                                         Sq, Skv, Skv, 0.125, ws.data_ptr(), ws.numel(), qs, sp, stream)

        def timeit(qs, sp):
            for _ in range(3):
                assert run(qs, sp) == 0
            evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                   for _ in range(a.reps)]
            for e0, e1 in evs:
                e0.record()
                run(qs, sp)
                e1.record()
            torch.cuda.synchronize()
            ts = sorted(e0.elapsed_time(e1) * 1000 for e0, e1 in evs)
            return ts[len(ts) // 2]

        th = timeit(0, 0)
        best = (th, "heur")
        allp = {}
        ktiles = (Skv + 63) // 64
        for qs in (1, 2):
            for sp in (1, 2, 3, 4, 6, 8, 12, 16):
                if sp > ktiles:
                    continue
                t = timeit(qs, sp)
                allp[f"q{qs}/s{sp}"] = round(t, 1)
                if t < best[0]:
                    best = (t, f"q{qs}/s{sp}")
        print(json.dumps(dict(Sq=Sq, H=Hh, Skv=Skv, B=B, heur_us=round(th, 2), heur_tflops=round(flops / th / 1e6, 1),
                              best_us=round(best[0], 2), best=best[1],
                              best_tflops=round(flops / best[0] / 1e6, 1), all=allp)), flush=True)


if __name__ == "__main__":
    main()
