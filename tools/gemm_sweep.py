#!/usr/bin/env python
"""GEMM sweep on the network's shapes at a given tile batch, with cold operands.

Every rep uses a different weight / activation buffer from a rotation whose total footprint
exceeds the 256 MiB Infinity Cache, so the weights stream from HBM as they do inside a denoise
step (an isolated loop over one buffer reads them from the MALL / L2 and flatters small tiles).
Compares the planner's choice, forced (tile, split) candidates and torch.matmul (hipBLASLt) on the
same rotation.  Prints one JSON line per shape.

    python tools/gemm_sweep.py --batch 1 8 64 [--sweep] [--shapes conv64,lin64ff1]
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

# name: (mode, side (output H=W), N, K or Cin for convs, Kx)   mode 0 dense, 1 conv3, 2 conv3 s2, 3 conv3 up
SHAPES = {
    "lin64proj": (0, 64, 320, 320, 0), "lin64qkv": (0, 64, 960, 320, 0), "lin64ff1": (0, 64, 2560, 320, 0),
    "lin64ff2": (0, 64, 320, 1280, 0), "conv64": (1, 64, 320, 320, 0), "conv64cat": (1, 64, 320, 320, 640),
    "lin32proj": (0, 32, 640, 640, 0), "lin32ff1": (0, 32, 5120, 640, 0), "lin32ff2": (0, 32, 640, 2560, 0),
    "conv32": (1, 32, 640, 640, 0), "lin16proj": (0, 16, 1280, 1280, 0), "lin16ff1": (0, 16, 10240, 1280, 0),
    "lin16ff2": (0, 16, 1280, 5120, 0), "conv16": (1, 16, 1280, 1280, 0), "conv8": (1, 8, 1280, 1280, 0),
    "conv8cat": (1, 8, 1280, 1280, 1280), "down32": (2, 32, 320, 320, 0), "up64": (3, 64, 640, 640, 0),
    "lin32qkv": (0, 32, 1920, 640, 0), "lin16qkv": (0, 16, 3840, 1280, 0), "lin8proj": (0, 8, 1280, 1280, 0),
    "conv32in": (1, 32, 640, 320, 0), "conv16in": (1, 16, 1280, 640, 0), "up32": (3, 32, 1280, 1280, 0),
    "up16": (3, 16, 1280, 1280, 0), "down16": (2, 16, 640, 640, 0), "down8": (2, 8, 1280, 1280, 0),
    "lin64ff1plain": (0, 64, 2560, 320, 0), "lin32ff1plain": (0, 32, 5120, 640, 0),  # (no GEGLU epilogue)
}
HALO_TILES = [(256, 64), (256, 128), (256, 160)]  # conv_halo_kernel (force_stages 9): stride-1 3x3, no Kx
HALO_SPLITS = [1, 2, 3, 4, 5, 6, 8, 10, 12, 16, 20]
TILES = [(64, 64), (64, 128), (128, 64), (128, 128), (128, 256), (256, 256), (128, 320), (256, 320),
         (-128, 320), (-256, 256), (-256, 128), (-128, 256), (-128, 128), (-64, 128), (-64, 64)]  # -bm: BK=32 ring
SPLITS = [1, 2, 3, 4, 6, 8]


class Rot:
    """A rotation of operand sets, > 256 MiB in total."""

    def __init__(self, mode, B, side, N, K, Kx, min_bytes=320 << 20):
        M = B * side * side
        if mode == 0:
            hin, C, Kt = side, K, K
        else:
            C = K
            hin = {1: side, 2: 2 * side, 3: side // 2}[mode]
            Kt = 9 * C
        a_el = B * hin * hin * C
        w_el = N * (Kt + Kx)
        per = 2 * (a_el + w_el + M * Kx + M * N)
        n = max(2, min(64, min_bytes // max(per, 1) + 1))
        self.sets = []
        for _ in range(n):
            a = (torch.randn(a_el, device="cuda") * 0.5).to(torch.bfloat16)
            w = (torch.randn(w_el, device="cuda") * 0.02).to(torch.bfloat16)
            x = (torch.randn(max(M * Kx, 1), device="cuda") * 0.5).to(torch.bfloat16)
            o = torch.empty(M * N, device="cuda", dtype=torch.bfloat16)
            self.sets.append((a, w, x, o))
        self.mode, self.B, self.side, self.N, self.K, self.Kx, self.M, self.C, self.hin, self.Kt = \
            mode, B, side, N, K, Kx, M, C, hin, Kt
        self.geglu = False
        self.bias = torch.randn(N, device="cuda")
        self.part = torch.empty(32 << 20, device="cuda")
        self.sem = torch.zeros(1 << 16, device="cuda", dtype=torch.int32)

    def desc(self, i, bm=0, bn=0, s=0, sem=True, halo=False):
        a, w, x, o = self.sets[i % len(self.sets)]
        d = _lib.GemmDesc()
        d.M, d.N, d.amode, d.alpha = self.M, self.N, self.mode, 1.0
        d.Wt, d.ldw, d.out, d.ldo, d.bias = w.data_ptr(), self.Kt + self.Kx, o.data_ptr(), self.N, self.bias.data_ptr()
        d.partial, d.partial_cap = self.part.data_ptr(), self.part.numel()
        d.A, d.K = a.data_ptr(), self.Kt
        d.lda = self.C
        if self.mode:
            d.C, d.Bn, d.H, d.W, d.Ho, d.Wo = self.C, self.B, self.hin, self.hin, self.side, self.side
            d.rows_per_b = self.side * self.side
        if self.Kx:
            d.X, d.ldx, d.Kx = x.data_ptr(), self.Kx, self.Kx
        d.force_bm, d.force_bn, d.force_splits = bm, bn, s
        if self.geglu:  # the FF proj's epilogue (x * gelu(gate) pairs, N / 2 output columns)
            d.act, d.ldo = 2, self.N // 2
        if halo:
            d.force_stages = 9
        if sem:
            d.tile_sem, d.sem_cap = self.sem.data_ptr(), self.sem.numel()
        return d


def time_fn(fn, reps):
    st = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for i in range(3):
        fn(i)
    for i, (a, b) in enumerate(st):
        a.record()
        fn(i)
        b.record()
    torch.cuda.synchronize()
    ts = sorted(a.elapsed_time(b) * 1000 for a, b in st)
    return ts[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, nargs="+", default=[1])
    ap.add_argument("--shapes", default="")
    ap.add_argument("--sweep", action="store_true")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--tiles", default="", help="restrict the sweep to these tiles, e.g. 64x64,128x320")
    a = ap.parse_args()
    L = _lib.lib()
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    names = a.shapes.split(",") if a.shapes else list(SHAPES)
    for B in a.batch:
        tot = {"plan": 0.0, "best": 0.0, "blas": 0.0}
        for nm in names:
            mode, side, N, K, Kx = SHAPES[nm]
            r = Rot(mode, B, side, N, K, Kx)
            r.geglu = nm.endswith("ff1")  # the planner's plan and every candidate run the GEGLU epilogue (tickets given)
            flops = 2.0 * r.M * N * (r.Kt + Kx)

            def run(d):
                rc = L.tair_k_gemm(ctypes.byref(d), stream)
                assert rc == 0, L.tair_last_error()

            descs = [r.desc(i) for i in range(len(r.sets))]
            t_plan = time_fn(lambda i: run(descs[i % len(descs)]), a.reps)
            best = (t_plan, "plan")
            if a.sweep:
                tiles = [tuple(int(v) for v in t.split("x")) for t in a.tiles.split(",")] if a.tiles else TILES
                for bm, bn in tiles:
                    if bn > 128 and (r.M * N) / (abs(bm) * bn) < 64:
                        continue
                    for s in SPLITS:
                        if s > (r.Kt + Kx) // 64 // 2 and s > 1:
                            continue
                        for sem in ([False, True] if s > 1 else [False]):
                            ds = [r.desc(i, bm, bn, s, sem) for i in range(len(r.sets))]
                            t = time_fn(lambda i: run(ds[i % len(ds)]), a.reps)
                            if t < best[0]:
                                best = (t, f"{bm}x{bn}/s{s}{'/sem' if sem else ''}")
                if mode == 1 and not Kx and side in (16, 32, 64) and (r.M % 256) == 0:
                    for bm, bn in HALO_TILES:
                        if bn == 64 and side != 64:
                            continue
                        for s in HALO_SPLITS:
                            if s > K // 64:
                                continue
                            ds = [r.desc(i, bm, bn, s, False, True) for i in range(len(r.sets))]
                            try:
                                t = time_fn(lambda i: run(ds[i % len(ds)]), a.reps)
                            except AssertionError:
                                continue
                            if t < best[0]:
                                best = (t, f"halo{bm}x{bn}/s{s}")
            t_blas = None
            if mode == 0:
                mats = [(s_[0][:r.M * K].view(r.M, K), s_[1][:N * K].view(N, K)) for s_ in r.sets]
                t_blas = time_fn(lambda i: torch.matmul(mats[i % len(mats)][0], mats[i % len(mats)][1].t()), a.reps)
            tot["plan"] += t_plan
            tot["best"] += best[0]
            tot["blas"] += t_blas if t_blas else best[0]
            print(json.dumps(dict(B=B, shape=nm, M=r.M, N=N, K=r.Kt + Kx, plan_us=round(t_plan, 2),
                                  plan_tf=round(flops / t_plan / 1e6, 1), best=best[1], best_us=round(best[0], 2),
                                  best_tf=round(flops / best[0] / 1e6, 1),
                                  blas_us=round(t_blas, 2) if t_blas else None,
                                  blas_tf=round(flops / t_blas / 1e6, 1) if t_blas else None)), flush=True)
            del r
            torch.cuda.empty_cache()
        print(json.dumps(dict(B=B, totals_us={k: round(v, 1) for k, v in tot.items()})), flush=True)


if __name__ == "__main__":
    main()
