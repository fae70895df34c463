#!/usr/bin/env python
"""Time the stride-1 3x3 conv GEMMs of the UNet (ResBlock conv1 / identity-skip conv2 shapes) at a batch.

Prints one JSON line per shape: the heuristic plan's time (HIP events, median of --reps) and, with
--no-epilogue, the main loop alone (probe bit 1).  Run it once with TAIR_HALO=0 and once without to
compare the halo-tile kernel against the implicit-GEMM tile kernels; --force BMxBN/S/ST forces a plan.
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

# (side, C_in, C_out): encoder / decoder ResBlock convs of SD-2.1 at a 64x64 latent (unet.py:203-223)
SHAPES = [(64, 320, 320), (64, 640, 320), (64, 960, 320),
          (32, 320, 640), (32, 640, 640), (32, 960, 640), (32, 1280, 640), (32, 1920, 640),
          (16, 640, 1280), (16, 1280, 1280), (16, 1920, 1280), (16, 2560, 1280),
          (8, 1280, 1280), (8, 2560, 1280)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, nargs="+", default=[1, 16, 64])
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--no-epilogue", action="store_true")
    ap.add_argument("--force", default="", help="BMxBN/S/ST, e.g. 256x64/1/9 (halo)")
    ap.add_argument("--tag", default=os.environ.get("TAIR_HALO", "default"))
    ap.add_argument("--gn", action="store_true", help="GroupNorm+SiLU on load (GemmArgs.gn_st, synthetic stats)")
    ap.add_argument("--only", default="", help="side,C,N: time just this shape")
    ap.add_argument("--ablate", type=int, default=0,
                    help="halo-kernel ablation bits (timing only): 8 no weight DMA, 16 no MFMA, 32 no loop barrier")
    a = ap.parse_args()
    L = _lib.lib()
    torch.manual_seed(0)
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    maxb = max(a.batch)
    act = (torch.randn(maxb * 64 * 64 * 960, device="cuda") * 0.5).to(torch.bfloat16)
    wts = (torch.randn(1280 * 9 * 2560, device="cuda") * 0.02).to(torch.bfloat16)
    out = torch.empty(maxb * 64 * 64 * 320 + (1 << 20), device="cuda", dtype=torch.bfloat16)
    bias = torch.randn(4096, device="cuda")
    part = torch.empty(64 << 20, device="cuda")
    G = 32
    gst = torch.zeros(8, maxb * G * 2, device="cuda", dtype=torch.float64)
    gst[0, 1::2] = 64 * 64 * 80.0  # sum of squares: var ~ 1 for every group at any (side, C)
    gam = torch.rand(2560, device="cuda") + 0.5
    bet = torch.randn(2560, device="cuda")
    total = {}
    for B in a.batch:
        for side, C, N in ([tuple(int(v) for v in a.only.split(","))] if a.only else SHAPES):
            M = B * side * side
            if M * C > act.numel() or M * N > out.numel():
                continue
            d = _lib.GemmDesc()
            d.M, d.N, d.K, d.amode = M, N, 9 * C, 1
            d.A, d.lda, d.C = act.data_ptr(), C, C
            d.Bn, d.H, d.W, d.Ho, d.Wo = B, side, side, side, side
            d.rows_per_b = side * side
            d.Wt, d.ldw = wts.data_ptr(), 9 * C
            d.alpha = 1.0
            d.bias = bias.data_ptr()
            d.out, d.ldo = out.data_ptr(), N
            d.partial, d.partial_cap = part.data_ptr(), part.numel()
            d.probe = (2 if a.no_epilogue else 0) | a.ablate
            if a.gn:
                d.gn_st, d.gn_rs, d.gn_G, d.gn_eps = gst.data_ptr(), maxb * G * 2, G, 1e-5
                d.gn_gamma, d.gn_beta, d.gn_silu = gam.data_ptr(), bet.data_ptr(), 1
            if a.force:
                t, s, st = a.force.split("/")
                d.force_bm, d.force_bn = (int(x) for x in t.split("x"))
                d.force_splits, d.force_stages = int(s), int(st)
            if L.tair_k_gemm(ctypes.byref(d), stream) != 0:
                print(json.dumps({"B": B, "side": side, "C": C, "N": N, "error": L.tair_last_error().decode()}))
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
            tf = 2.0 * M * N * 9 * C / us / 1e6
            total[B] = total.get(B, 0.0) + us
            print(json.dumps({"tag": a.tag, "ablate": a.ablate, "B": B, "side": side, "C": C, "N": N, "us": round(us, 1),
                              "tflops": round(tf, 1)}), flush=True)
    print(json.dumps({"tag": a.tag, "total_us": {k: round(v, 1) for k, v in total.items()}}), flush=True)


if __name__ == "__main__":
    main()
