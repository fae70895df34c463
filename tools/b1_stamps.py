#!/usr/bin/env python
"""Where a B = 1 GEMM launch spends its time, from in-kernel phase stamps (a library built with
-DTAIR_STAMPS=1: `python -m tair_amd.build --variant stamps -D TAIR_STAMPS=1`, run with
TAIR_LIB_VARIANT=stamps).  Lane 0 of every workgroup records s_memrealtime (100 MHz) at: 0 entry, 1 prologue
DMA issued, 2 first K-tile landed (after its barrier), 3 main loop done, 4 epilogue start (after the
in-kernel split-K combine), 5 accumulators staged in LDS, 6 items stored, 7 exit.  Per launch: the
quantiles over workgroups of each phase (us) and of the entry / exit times relative to the first entry.

    TAIR_LIB_VARIANT=stamps python tools/b1_stamps.py [--shapes lin64proj,conv16] [--variants plan,halo256x64/s5]
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

from b1_probe import parse_variant  # noqa: E402
from gemm_sweep import SHAPES, Rot  # noqa: E402
from tair_amd import _lib  # noqa: E402

PHASES = [("prologue", 0, 1), ("first_data", 1, 2), ("loop", 2, 3), ("combine", 3, 4), ("stage", 4, 5),
          ("items", 5, 6), ("flush", 6, 7)]


def q(v, f):
    v = sorted(v)
    return round(v[min(len(v) - 1, int(f * len(v)))], 2) if v else None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="lin64proj,lin32proj,lin16proj,lin64qkv,conv64,conv16,conv8")
    ap.add_argument("--variants", default="plan")
    a = ap.parse_args()
    L = _lib.lib()
    s = torch.cuda.Stream()
    sp = ctypes.c_void_p(s.cuda_stream)
    st = torch.zeros(65536 * 8 + 4 * 64 * 4, dtype=torch.int64, device="cuda")
    for nm in a.shapes.split(","):
        mode, side, N, K, Kx = SHAPES[nm]
        r = Rot(mode, 1, side, N, K, Kx)
        for vs in a.variants.split(","):
            v = parse_variant(vs)
            if v["halo"] and (mode != 1 or Kx or side not in (16, 32, 64) or (v["bn"] == 64 and side != 64)):
                continue
            ds = []
            for i in range(len(r.sets)):
                d = r.desc(i, v["bm"], v["bn"], v["s"], v["sem"], v["halo"])
                d.probe = v["probe"]
                if v["deep"]:
                    d.force_stages = 100 + v["deep"]
                ds.append(d)
            with torch.cuda.stream(s):
                for d in ds:  # one pass over the rotation: cold weights for the stamped launch
                    assert L.tair_k_gemm(ctypes.byref(d), sp) == 0, L.tair_last_error().decode()
                st.zero_()
                d = ds[0]
                d.stamps = st.data_ptr()
                assert L.tair_k_gemm(ctypes.byref(d), sp) == 0, L.tair_last_error().decode()
                d.stamps = None
            s.synchronize()
            allst = st.cpu()
            t = allst[:65536 * 8].view(-1, 8)
            rows = t[t[:, 0] > 0].tolist()
            loop = allst[65536 * 8:65536 * 8 + 4 * 64 * 4].view(4, 64, 4).tolist()  # TAIR_STAMPS >= 2 builds
            if not rows:
                print(json.dumps(dict(shape=nm, variant=vs, error="no stamps (not a TAIR_STAMPS build?)")))
                continue
            t0 = min(rw[0] for rw in rows)
            us = lambda x: x / 100.0  # 100 MHz ticks -> us
            out = dict(shape=nm, variant=vs, wgs=len(rows),
                       entry=[q([us(rw[0] - t0) for rw in rows], f) for f in (0.5, 0.9, 1.0)],
                       exit=[q([us(rw[7] - t0) for rw in rows if rw[7]], f) for f in (0.1, 0.5, 0.9, 1.0)])
            for name, i, j in PHASES:
                vals = [us(rw[j] - rw[i]) for rw in rows if rw[i] and rw[j] and rw[j] >= rw[i]]
                if vals:
                    out[name] = [q(vals, 0.5), q(vals, 0.9)]
            its = [r for r in loop[0] if r[0]]
            if len(its) > 1:  # block 0's main-loop iterations: wait+barrier / issue / MFMA segments, period (us)
                seg = lambda a, b: [round((r[b] - r[a]) / 100.0, 2) for r in its if r[b] and r[a]]
                out["it_wait"] = seg(0, 1)[:24]
                out["it_issue"] = seg(1, 2)[:24]
                out["it_mfma"] = seg(2, 3)[:24]
                out["it_period"] = [round((its[i + 1][0] - its[i][0]) / 100.0, 2) for i in range(len(its) - 1)][:24]
            ib = loop[0]  # block 0, thread 0: epilogue items (slots 48 + 2 pass + 8 item): operands, epilogue8, end
            segs = []
            for slot in range(48, 64):
                r0 = ib[slot]
                if r0[0] and r0[1] and r0[2]:
                    segs.append([slot, round((r0[1] - r0[0]) / 100.0, 2), round((r0[2] - r0[1]) / 100.0, 2)])
            if segs:
                out["items_seg"] = segs
            print(json.dumps(out), flush=True)
        del r
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
