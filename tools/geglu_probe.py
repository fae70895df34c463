#!/usr/bin/env python
"""Where the batched GEGLU-in linear (FF proj, attention.py:54-70 / the product's LayerNorm-folded FF-in GEMM)
spends its time: the planner's plan vs forced tiles, each with the product's epilogue (LayerNorm fold + bias +
GEGLU) and with the GemmArgs measurement probes (e1: values formed, not stored; e2: no epilogue).

    python tools/geglu_probe.py [--batch 64] [--levels 64,32,16] [--tiles 0x0,256x256,e1:256x256,...]

Tile syntax: [eP:][kS:]BMxBN[sSPLITS]; --plain --nmul 1 [--res] [--rst] for proj_in / out-projection shapes  (P = GemmArgs.probe, S = force_stages, e.g. k4 = the phase kernel).
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

LEVELS = {64: 320, 32: 640, 16: 1280, 8: 1280}  # latent side -> channels (SD-2.1 UNet)


def parse(t):
    probe = stages = 0
    sp = 1
    while t[0] in "ek" and ":" in t:
        tag, t = t.split(":", 1)
        if tag[0] == "e":
            probe = int(tag[1:])
        else:
            stages = int(tag[1:])
    if "s" in t:
        t, s = t.split("s")
        sp = int(s)
    bm, bn = (int(v) for v in t.split("x"))
    return bm, bn, sp, probe, stages


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--levels", default="64,32,16")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--tiles", default="0x0,256x256,e1:256x256,e2:256x256")
    ap.add_argument("--noln", action="store_true", help="drop the LayerNorm fold (bias + GEGLU only)")
    ap.add_argument("--plain", action="store_true", help="no GEGLU: the full N columns stored")
    ap.add_argument("--nmul", type=int, default=8, help="N = nmul x C (8: GEGLU-in, 1: proj_in / out-projections)")
    ap.add_argument("--res", action="store_true", help="residual added in place (plain only)")
    ap.add_argument("--rst", action="store_true", help="LayerNorm row statistics of the output (plain only)")
    a = ap.parse_args()
    L = _lib.lib()
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    torch.manual_seed(0)
    for side in (int(s) for s in a.levels.split(",")):
        C = LEVELS[side]
        M, K, N = a.batch * side * side, C, a.nmul * C
        x = (torch.randn(M, K, device="cuda") * 0.5).to(torch.bfloat16)
        w = (torch.randn(N, K, device="cuda") * 0.05).to(torch.bfloat16)
        out = torch.empty(M, N if a.plain else N // 2, device="cuda", dtype=torch.bfloat16)
        bias = torch.randn(N, device="cuda") * 0.1
        xf = x.float()
        mean, var = xf.mean(1, dtype=torch.float64), xf.var(1, unbiased=False).double()
        lnst = torch.stack([mean * K, (var + mean * mean) * K], 1).contiguous()
        lncs = w.float().sum(1).contiguous()
        del xf
        flops = 2.0 * M * N * K
        row = {"B": a.batch, "side": side, "M": M, "N": N, "K": K}
        for t in a.tiles.split(","):
            bm, bn, sp, probe, stages = parse(t)
            d = _lib.GemmDesc()
            d.M, d.N, d.K, d.amode, d.alpha = M, N, K, 0, 1.0
            d.A, d.lda, d.Wt, d.ldw = x.data_ptr(), K, w.data_ptr(), K
            d.out, d.ldo, d.bias = out.data_ptr(), out.shape[1], bias.data_ptr()
            d.act = 0 if a.plain else 2
            if not a.noln:
                d.lnst, d.lncs, d.ln_c, d.ln_eps = lnst.data_ptr(), lncs.data_ptr(), float(K), 1e-5
            d.probe = probe
            if a.res:
                d.res, d.ld_res = out.data_ptr(), out.shape[1]
            if a.rst:
                rst = torch.zeros(M, 2, device="cuda", dtype=torch.float64)
                d.rst = rst.data_ptr()
            d.force_bm, d.force_bn, d.force_splits, d.force_stages = bm, bn, (sp if bm else 0), stages
            if bm == 0:
                pb, pn, ps, pk = ctypes.c_int(), ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
                if L.tair_k_gemm_plan(ctypes.byref(d), ctypes.byref(pb), ctypes.byref(pn), ctypes.byref(ps),
                                      ctypes.byref(pk)) == 0:
                    row["plan_cfg"] = f"{pb.value}x{pn.value}/s{ps.value}/k{pk.value}"
            rc = L.tair_k_gemm(ctypes.byref(d), stream)
            if rc != 0:
                row[t] = "refused: " + L.tair_last_error().decode()
                continue
            evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.reps)]
            for _ in range(2):
                L.tair_k_gemm(ctypes.byref(d), stream)
            for e0, e1 in evs:
                e0.record()
                L.tair_k_gemm(ctypes.byref(d), stream)
                e1.record()
            torch.cuda.synchronize()
            ts = sorted(e0.elapsed_time(e1) * 1000 for e0, e1 in evs)
            us = ts[len(ts) // 2]
            row[t] = [round(us, 1), round(flops / us / 1e6)]
        print(json.dumps(row), flush=True)
        del x, w, out, lnst, lncs
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
