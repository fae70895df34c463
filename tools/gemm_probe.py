#!/usr/bin/env python
"""Probe where a large-M GEMM spends its time: the planner's choice vs forced tiles, with and without
the epilogue extras (GEGLU, residual), on the batched network's linear / conv shapes.

python tools/gemm_probe.py [--batch 16] [--reps 10]
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
sys.path.insert(0, os.path.join(ROOT, "tools"))

from gemm_bench import make_desc, time_desc  # noqa: E402
from tair_amd import _lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--tiles", default="0x0,64x64,128x128,128x256,256x256,128x320,256x320")
    ap.add_argument("--shapes", default="")
    a = ap.parse_args()
    L = _lib.lib()
    B = a.batch
    M64 = B * 4096
    shapes_b1 = [  # the B = 1 network's weight-streaming shapes (M = B * H * W at 8^2 .. 64^2)
        ("conv8", 1, 64, 1280, 11520, 0, 0), ("conv16", 1, 256, 1280, 11520, 0, 0),
        ("conv32", 1, 1024, 640, 5760, 0, 0), ("conv64", 1, 4096, 320, 2880, 0, 0),
        ("up64", 3, 4096, 640, 5760, 0, 0), ("ff1_16", 0, 256, 10240, 1280, 2, 0),
        ("ff2_16", 0, 256, 1280, 5120, 0, 1), ("proj16", 0, 256, 1280, 1280, 0, 1),
        ("ff1_32", 0, 1024, 5120, 640, 2, 0), ("ff2_32", 0, 1024, 640, 2560, 0, 1),
        ("proj32", 0, 1024, 640, 640, 0, 1), ("proj64", 0, 4096, 320, 320, 0, 1),
    ]
    shapes = [  # name, mode, M, N, K, act, res
        ("proj64", 0, M64, 320, 320, 0, 1),
        ("qkv64", 0, M64, 960, 320, 0, 0),
        ("ff1_64", 0, M64, 2560, 320, 2, 0),
        ("ff1_64_noact", 0, M64, 2560, 320, 0, 0),
        ("ff2_64", 0, M64, 320, 1280, 0, 1),
        ("ff1_32", 0, M64 // 4, 5120, 640, 2, 0),
        ("proj32", 0, M64 // 4, 640, 640, 0, 1),
        ("qkv32", 0, M64 // 4, 1920, 640, 0, 0),
        ("ff1_16", 0, M64 // 16, 10240, 1280, 2, 0),
        ("conv64", 1, M64, 320, 2880, 0, 0),
        ("conv32", 1, M64 // 4, 640, 5760, 0, 0),
        # the 16^2 / 8^2 levels (small grids at B = 16: the planner splits K)
        ("conv16", 1, M64 // 16, 1280, 11520, 0, 0),
        ("conv8", 1, M64 // 64, 1280, 11520, 0, 0),
        ("ff2_16", 0, M64 // 16, 1280, 5120, 0, 1),
        ("proj16", 0, M64 // 16, 1280, 1280, 0, 1),
        ("ff1_8", 0, M64 // 64, 10240, 1280, 2, 0),
        ("ff2_8", 0, M64 // 64, 1280, 5120, 0, 1),
    ]
    big = 96 << 20
    torch.manual_seed(0)
    bufs = {
        "a": (torch.randn(big, device="cuda") * 0.5).to(torch.bfloat16),
        "x": (torch.randn(big // 4, device="cuda") * 0.5).to(torch.bfloat16),
        "w": (torch.randn(16 << 20, device="cuda") * 0.02).to(torch.bfloat16),
        "out": torch.empty(big * 2, device="cuda", dtype=torch.bfloat16),
        "res": (torch.randn(big, device="cuda")).to(torch.bfloat16),
        "bias": torch.randn(65536, device="cuda"),
        "part": torch.empty(64 << 20, device="cuda"),
    }
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    # "p256x256": 4-phase kernel; "a5:p256x256" / "a6:..." its ablations (no DMA / no MFMA in the loop);
    # "64x64s8": forced split-K 8 (default 1)
    # "e1:..." / "e2:...": the GEMM's measurement probes (GemmArgs.probe: 1 no epilogue stores, 2 no
    # epilogue); "0x0" = the planner's tile
    def tile(t):
        abl, sp, probe = 0, 1, 0
        if t.startswith("e"):
            probe, t = int(t[1]), t[3:]
        if t.startswith("a"):
            abl, t = int(t[1]), t[3:]
        if "s" in t:
            t, sp = t.split("s")
            sp = int(sp)
        bm, bn = (int(v) for v in t.lstrip("p").split("x"))
        return (abl if abl else (4 if t.startswith("p") else 0), bm, bn, sp, probe)
    tiles = [tile(t) for t in a.tiles.split(",")]
    if a.batch == 1:
        shapes = shapes_b1
    if a.shapes:
        shapes = [s for s in shapes if s[0] in a.shapes.split(",")]
    for name, mode, M, N, K, act, res in shapes:
        flops = 2.0 * M * N * K
        # host-side bounds check of the operand buffers (an oversized shape would read past them)
        a_el = M * K if mode == 0 else (M * 4 if mode == 2 else M) * (K // 9)
        if a_el > bufs["a"].numel() or N * K > bufs["w"].numel() or M * N > bufs["out"].numel() or \
                (res and M * N > bufs["res"].numel()):
            print(json.dumps({"shape": name, "M": M, "N": N, "K": K, "skipped": "exceeds the probe buffers"}))
            continue
        row = {"shape": name, "M": M, "N": N, "K": K}
        for ph, bm, bn, sp, probe in tiles:
            d = make_desc(mode, M, N, K, 0, bufs, B=B)
            d.probe = probe
            d.act = act
            d.ldo = N // 2 if act == 2 else N
            if res:
                d.res, d.ld_res = bufs["res"].data_ptr(), N
            d.force_bm, d.force_bn, d.force_splits = bm, bn, sp if bm else 0
            d.force_stages = ph
            try:
                t = time_desc(L, d, a.reps, stream)
            except AssertionError:
                continue
            key = (f"k{ph}:" if ph else "") + f"{bm}x{bn}s{sp}" if bm else "plan"
            row[(f"e{probe}:" if probe else "") + key] = [round(t, 1), round(flops / t / 1e6)]
            if bm == 0:
                pb, pn, ps, pk = ctypes.c_int(), ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
                if L.tair_k_gemm_plan(ctypes.byref(d), ctypes.byref(pb), ctypes.byref(pn), ctypes.byref(ps),
                                      ctypes.byref(pk)) == 0:
                    row["plan_cfg"] = f"{pb.value}x{pn.value}/s{ps.value}/k{pk.value}"
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
