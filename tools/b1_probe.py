#!/usr/bin/env python
"""Per-launch GEMM cost at B = 1 measured the way the step graph runs it: N dependent launches of one
shape captured in a HIP graph (no host launch cost in the timing), operands rotated over > 256 MiB so
the weights stream from HBM as in a denoise step.  Variants: the planner's plan, forced (tile, splits,
in-kernel combine), halo tiles (force_stages 9), and the measurement probes (e1: values formed but not
stored, e2: no epilogue).

    python tools/b1_probe.py [--shapes lin64proj,conv8] [--variants plan,64x64/s1,e2:plan] [--n 40]
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

from gemm_sweep import SHAPES, Rot  # noqa: E402
from tair_amd import _lib  # noqa: E402

DEFAULT_VARIANTS = "plan,e1:plan,e2:plan,64x64/s1,64x64/s2/sem,64x128/s1,128x64/s1,128x128/s1,64x64/s4"


def parse_variant(v):
    """'[eP:][dS:]plan' | '[eP:][dS:]BMxBN/sS[/sem]' | '[eP:]haloBMxBN/sS' -> dict (eP: probe bits P, dS: deep
    ring of S stages)"""
    probe, deep = 0, 0
    while ":" in v:
        pre, v = v.split(":", 1)
        if pre.startswith("e"):
            probe = int(pre[1:])
        elif pre.startswith("d"):  # deep-ring tile kernel with this many stages
            deep = int(pre[1:])
    if v == "plan":
        return dict(probe=probe, bm=0, bn=0, s=0, sem=True, halo=False, deep=deep)
    halo = v.startswith("halo")
    parts = v.replace("halo", "").split("/")
    bm, bn = (int(x) for x in parts[0].split("x"))
    s = int(parts[1][1:]) if len(parts) > 1 else 1
    sem = "sem" in parts
    return dict(probe=probe, bm=bm, bn=bn, s=s, sem=sem, halo=halo, deep=deep)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="")
    ap.add_argument("--variants", default=DEFAULT_VARIANTS)
    ap.add_argument("--n", type=int, default=40, help="launches per graph")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--warm", action="store_true", help="two operand sets only: weights stay in L2 / the MALL")
    a = ap.parse_args()
    L = _lib.lib()
    names = a.shapes.split(",") if a.shapes else list(SHAPES)
    variants = a.variants.split(",")
    s = torch.cuda.Stream()
    sp = ctypes.c_void_p(s.cuda_stream)
    for nm in names:
        mode, side, N, K, Kx = SHAPES[nm]
        r = Rot(mode, 1, side, N, K, Kx, min_bytes=1 if a.warm else 320 << 20)
        flops = 2.0 * r.M * N * (r.Kt + Kx)
        row = dict(shape=nm, M=r.M, N=N, K=r.Kt + Kx)
        pb, pn, ps, pk = ctypes.c_int(), ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        d0 = r.desc(0, 0, 0, 0, True)
        if L.tair_k_gemm_plan(ctypes.byref(d0), ctypes.byref(pb), ctypes.byref(pn), ctypes.byref(ps),
                              ctypes.byref(pk)) == 0:
            row["plan"] = f"{pb.value}x{pn.value}/s{ps.value}/k{pk.value}"
        for vs in variants:
            v = parse_variant(vs)
            if v["halo"] and (mode != 1 or Kx or side not in (16, 32, 64)):
                continue
            ds = []
            for i in range(len(r.sets)):
                d = r.desc(i, v["bm"], v["bn"], v["s"], v["sem"], v["halo"])
                d.probe = v["probe"]
                if v["deep"]:
                    d.force_stages = 100 + v["deep"]
                ds.append(d)
            try:
                with torch.cuda.stream(s):
                    for d in ds[:2]:  # eager first: kernel attributes / validation outside the capture
                        assert L.tair_k_gemm(ctypes.byref(d), sp) == 0, L.tair_last_error().decode()
                s.synchronize()
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, stream=s):
                    for i in range(a.n):
                        assert L.tair_k_gemm(ctypes.byref(ds[i % len(ds)]), sp) == 0
            except AssertionError as e:
                row[vs] = f"err {str(e)[:60]}"
                continue
            g.replay()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            ts = []
            for _ in range(a.reps):
                e0.record(s)
                with torch.cuda.stream(s):
                    g.replay()
                e1.record(s)
                e1.synchronize()
                ts.append(e0.elapsed_time(e1) * 1000.0 / a.n)
            ts.sort()
            t = ts[len(ts) // 2]
            row[vs] = [round(t, 2), round(flops / t / 1e6, 1)]
            del g
        print(json.dumps(row), flush=True)
        del r
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
