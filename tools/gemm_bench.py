#!/usr/bin/env python
"""Sweep the MFMA GEMM kernel's tile / split-K configurations over the network's GEMM shapes.

Shapes come from a per-launch profile CSV (bench.py --profile-only with TAIR_PROFILE_CSV=...).
For each unique (mode, M, N, K, Kx) it times the heuristic plan and every forced (tile, splits)
candidate with HIP events (median of N reps) and prints/saves the best.
"""
from __future__ import annotations

import argparse
import csv
import ctypes
import json
import math
import os
import re
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from tair_amd import _lib  # noqa: E402

TILES = [(128, 128), (64, 128), (128, 64), (64, 64)]
SPLITS = [1, 2, 3, 4, 5, 6, 8, 10, 12, 16]
STAGES = [3, 4, 6, 8]  # 6: 64-row tiles only; 8: 64x64 only (the launcher maps others down)


def shapes_from_csv(path):
    out = {}
    for r in csv.DictReader(open(path)):
        m = re.match(r"gemm mode=(\d+) M=(\d+) N=(\d+) K=(\d+) Kx=(\d+)", r["tag"])
        if not m:
            continue
        key = tuple(int(x) for x in m.groups())
        out.setdefault(key, 0)
        out[key] += 1
    return out


def make_desc(mode, M, N, K, Kx, bufs, B=1):
    d = _lib.GemmDesc()
    d.M, d.N, d.amode = M, N, mode
    d.alpha = 1.0
    d.Wt = bufs["w"].data_ptr()
    d.out = bufs["out"].data_ptr()
    d.ldo = N
    d.bias = bufs["bias"].data_ptr()
    d.partial = bufs["part"].data_ptr()
    d.partial_cap = bufs["part"].numel()
    if mode == 0:
        d.K, d.A, d.lda = K, bufs["a"].data_ptr(), K
        d.ldw = K + Kx
    else:
        C = K // 9
        side = int(round(math.sqrt(M // B)))
        if mode == 1:
            hin = side
        elif mode == 2:
            hin = 2 * side
        elif mode == 3:
            hin = side // 2
        else:
            raise ValueError(mode)
        d.K, d.A, d.lda, d.C = K, bufs["a"].data_ptr(), C, C
        d.Bn, d.H, d.W, d.Ho, d.Wo = B, hin, hin, side, side
        d.rows_per_b = side * side
        d.ldw = K + Kx
        if Kx:
            d.X, d.ldx, d.Kx = bufs["x"].data_ptr(), Kx, Kx
    return d


def time_desc(L, d, reps, stream):
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for _ in range(3):
        assert L.tair_k_gemm(ctypes.byref(d), stream) == 0, L.tair_last_error()
    ts = []
    for a, b in evs:
        a.record()
        L.tair_k_gemm(ctypes.byref(d), stream)
        b.record()
    torch.cuda.synchronize()
    ts = sorted(a.elapsed_time(b) * 1000 for a, b in evs)
    return ts[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--reps", type=int, default=15)
    ap.add_argument("--out", default=None)
    ap.add_argument("--sweep", action="store_true", help="try every tile/split candidate")
    a = ap.parse_args()
    L = _lib.lib()
    shapes = shapes_from_csv(a.csv)
    torch.manual_seed(0)
    big = 64 << 20
    bufs = {
        "a": (torch.randn(big, device="cuda") * 0.5).to(torch.bfloat16),
        "x": (torch.randn(big // 4, device="cuda") * 0.5).to(torch.bfloat16),
        "w": (torch.randn(big, device="cuda") * 0.02).to(torch.bfloat16),
        "out": torch.empty(big, device="cuda", dtype=torch.bfloat16),
        "bias": torch.randn(65536, device="cuda"),
        "part": torch.empty(16 << 20, device="cuda"),
    }
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    results = []
    tot_h = tot_b = 0.0
    for (mode, M, N, K, Kx), cnt in sorted(shapes.items(), key=lambda kv: -kv[0][1] * kv[0][2] * kv[0][3]):
        if mode == 4:
            continue
        flops = 2.0 * M * N * (K + Kx)
        d = make_desc(mode, M, N, K, Kx, bufs)
        th = time_desc(L, d, a.reps, stream)
        best = (th, "heur")
        if a.sweep:
            for st in STAGES:
                for bm, bn in TILES:
                    if (st >= 6 and bm != 64) or (st == 8 and bn != 64):
                        continue
                    for s in SPLITS:
                        if s > (K + Kx) // 64:
                            continue
                        d.force_bm, d.force_bn, d.force_splits, d.force_stages = bm, bn, s, st
                        t = time_desc(L, d, a.reps, stream)
                        if t < best[0]:
                            best = (t, f"{bm}x{bn}/s{s}/st{st}")
            d.force_bm = d.force_bn = d.force_splits = d.force_stages = 0
        tot_h += th * cnt
        tot_b += best[0] * cnt
        rec = dict(mode=mode, M=M, N=N, K=K, Kx=Kx, count=cnt, heur_us=round(th, 2),
                   heur_tflops=round(flops / th / 1e6, 1), best_us=round(best[0], 2),
                   best=best[1], best_tflops=round(flops / best[0] / 1e6, 1))
        results.append(rec)
        print(json.dumps(rec), flush=True)
    print(json.dumps({"total_heur_us": round(tot_h, 1), "total_best_us": round(tot_b, 1)}), flush=True)
    if a.out:
        json.dump(results, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
