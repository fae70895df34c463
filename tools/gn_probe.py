#!/usr/bin/env python
"""Bandwidth of the GroupNorm(+SiLU) apply from producer statistics (tair_k_gn_apply_stats) on the network's
shapes at one batch: one-plane inputs (ResBlock conv1 output) and hi + lo residual-stream inputs.  Prints
µs and GB/s of the bytes the pass must move (read 1 or 2 bf16 planes, write 1)."""
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

SHAPES = [(64, 320), (64, 640), (64, 960), (32, 640), (32, 1280), (32, 1920), (16, 1280), (16, 2560), (8, 1280)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    L = _lib.lib()
    dev = "cuda"
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    B, G = a.batch, 32
    for side, C in SHAPES:
        HW = side * side
        for lo in (0, 1):
            x = torch.randn(B * HW, 2 * C, device=dev).to(torch.bfloat16)
            y = torch.empty(B * HW, C, device=dev, dtype=torch.bfloat16)
            st = torch.zeros(8, B * G * 2, device=dev, dtype=torch.float64)
            st[0, 1::2] = HW * (C // G) * 1.0
            g = torch.ones(C, device=dev)
            be = torch.zeros(C, device=dev)

            def run():
                return L.tair_k_gn_apply_stats(x.data_ptr(), 2 * C, C if lo else 0, B, HW, C, G, 1e-5, g.data_ptr(),
                                               be.data_ptr(), 1, st.data_ptr(), B * G * 2, y.data_ptr(), C, 0, stream)
            assert run() == 0
            evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.reps)]
            for e0, e1 in evs:
                e0.record()
                run()
                e1.record()
            torch.cuda.synchronize()
            us = sorted(e0.elapsed_time(e1) * 1000 for e0, e1 in evs)[a.reps // 2]
            nbytes = B * HW * C * 2 * (3 if lo else 2)
            print(json.dumps({"B": B, "side": side, "C": C, "lo": lo, "us": round(us, 1),
                              "GBps": round(nbytes / us / 1e3, 1)}), flush=True)


if __name__ == "__main__":
    main()
