#!/usr/bin/env python
"""Time the batched short-K linears (K <= 1280) of the UNet at one batch, heuristic plan vs forced tiles.

Shapes (M = B * side^2 tokens): per SpatialTransformer (attention.py:219-353) q|k|v (N = 3C, K = C), attn2 q and
the out-projections (N = C), GEGLU-in (N = 8C, K = C) and FF-out (N = C, K = 4C), proj_in / proj_out (N = C).
Prints one JSON line per (shape, plan): median HIP-event time of --reps launches and TF/s; --no-epilogue sets
probe bit 1 (main loop only).
"""
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


def shapes(side, C):
    return [("qkv", 3 * C, C), ("proj", C, C), ("ff1", 8 * C, C), ("ff2", C, 4 * C)]


LEVELS = [(64, 320), (32, 640), (16, 1280)]
PLANS = ["heur", "64x64/1/2", "64x128/1/2", "64x64/1/3", "128x64/1/3", "128x128/1/3", "128x256/1/3",
         "256x128/1/3", "256x160/1/3", "128x320/1/2"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--no-epilogue", action="store_true")
    ap.add_argument("--probe", type=int, default=-1, help="GemmArgs.probe bits (1: no stores, 2: no epilogue)")
    ap.add_argument("--plans", default=",".join(PLANS))
    a = ap.parse_args()
    L = _lib.lib()
    torch.manual_seed(0)
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    Mmax = a.batch * 64 * 64
    act = (torch.randn(Mmax * 1280, device="cuda") * 0.5).to(torch.bfloat16)
    wts = (torch.randn(10240 * 1280, device="cuda") * 0.02).to(torch.bfloat16)
    out = torch.empty(Mmax * 2560, device="cuda", dtype=torch.bfloat16)
    bias = torch.randn(16384, device="cuda")
    part = torch.empty(64 << 20, device="cuda")
    for side, C in LEVELS:
        M = a.batch * side * side
        for name, N, K in shapes(side, C):
            if M * K > act.numel() or M * N > out.numel() or N * K > wts.numel():
                continue
            for plan in a.plans.split(","):
                d = _lib.GemmDesc()
                d.M, d.N, d.K, d.amode = M, N, K, 0
                d.A, d.lda = act.data_ptr(), K
                d.Wt, d.ldw = wts.data_ptr(), K
                d.alpha = 1.0
                d.bias = bias.data_ptr()
                d.out, d.ldo = out.data_ptr(), N
                d.partial, d.partial_cap = part.data_ptr(), part.numel()
                d.probe = a.probe if a.probe >= 0 else (2 if a.no_epilogue else 0)
                if plan != "heur":
                    t, s, st = plan.split("/")
                    d.force_bm, d.force_bn = (int(x) for x in t.split("x"))
                    d.force_splits, d.force_stages = int(s), int(st)
                if L.tair_k_gemm(ctypes.byref(d), stream) != 0:
                    continue
                evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                       for _ in range(a.reps)]
                for _ in range(2):
                    L.tair_k_gemm(ctypes.byref(d), stream)
                for e0, e1 in evs:
                    e0.record()
                    L.tair_k_gemm(ctypes.byref(d), stream)
                    e1.record()
                torch.cuda.synchronize()
                ts = sorted(e0.elapsed_time(e1) * 1000 for e0, e1 in evs)
                us = ts[len(ts) // 2]
                print(json.dumps({"B": a.batch, "side": side, "op": name, "M": M, "N": N, "K": K, "plan": plan,
                                  "epi": not a.no_epilogue, "probe": int(d.probe), "us": round(us, 1),
                                  "tflops": round(2.0 * M * N * K / us / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
