#!/usr/bin/env python
"""Per-kernel PMC summary from rocprofv3 `--pmc ... --output-format csv` counter files.

    python tools/pmc_summary.py OUT.json DIR [DIR ...] [--launches CSV --steps N]

Each DIR holds one pass (rocprofv3 cannot split counters over passes, so FETCH_SIZE, WRITE_SIZE and
the MFMA-busy counters are collected in separate runs of the same command).  Per kernel name
(template arguments kept, parameter list dropped) it reports the dispatch count and the mean per
dispatch of every counter found, plus the derived HBM bytes:

* FETCH_SIZE / WRITE_SIZE are in KiB.  On gfx950 FETCH_SIZE counts exactly half of the bytes of a
  wide (16 B/lane) coalesced streaming read (MI355X_MICROARCH.md, HBM section), which is how every
  tair GEMM / GroupNorm / attention load is issued, so read bytes = 2 * 1024 * FETCH_SIZE.  WRITE_SIZE
  is exact for 16-B-per-lane stores: write bytes = 1024 * WRITE_SIZE.
* MFMA busy fraction = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 * 1024 SIMDs) per dispatch:
  SQ_VALU_MFMA_BUSY_CYCLES is summed over all SIMDs (256 CUs x 4), and rocprofv3 reports
  GRBM_GUI_ACTIVE summed over the 8 XCDs (MI355X_MICROARCH.md, "DVFS give-back"), so the kernel's
  elapsed cycles are GRBM_GUI_ACTIVE / 8.  (Round 1 divided by GRBM_GUI_ACTIVE itself: 8x low.)
"""
from __future__ import annotations

import collections
import csv
import glob
import json
import os
import re
import sys

N_SIMD = 256 * 4
N_XCD = 8


def short(name: str) -> str:
    name = re.sub(r"tair::\(anonymous namespace\)::", "", name)
    depth, out = 0, []
    for ch in name:  # drop the parameter list but keep template arguments
        if ch == "(" and depth == 0 and out:
            break
        depth += ch == "<"
        depth -= ch == ">"
        out.append(ch)
    return "".join(out).strip()


def load(dirs):
    # (dispatch id, pass dir) -> {kernel, counters}
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    names = {}
    for d in dirs:
        files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
        if not files:
            raise SystemExit(f"no counter_collection.csv under {d}")
        for f in files:
            for r in csv.DictReader(open(f)):
                key = (d, f, r["Dispatch_Id"])
                names[key] = short(r["Kernel_Name"])
                per[key][r["Counter_Name"]] += float(r["Counter_Value"])
    return per, names


KEY_RULES = [  # rocprofv3 kernel name (short form) -> the launch key of cldm.cpp's profile CSV
    (re.compile(r"gemm_tile_kernel<(\d+), (\d+), \d+, \d+, \d+, (\d+), (\d+)>"), lambda m: f"tile:{m[1]}x{m[2]}:{m[3]}:{m[4]}"),
    (re.compile(r"conv_halo_kernel<(\d+),"), lambda m: f"halo:256x{m[1]}:1:0"),
    (re.compile(r"gemm_ring_kernel<(\d+), (\d+), \d+, \d+, \d+, \d+, (\d+)>"), lambda m: f"ring:{m[1]}x{m[2]}:{m[3]}:0"),
    (re.compile(r"gemm_phase_kernel<(\d+), (\d+)"), lambda m: f"phase:256x{m[1]}:{m[2]}:0"),
    (re.compile(r"gemm_kernel<(\d+), (\d+), (\d+)>"), lambda m: f"reg:{m[1]}x{m[2]}:{m[3]}:0"),
    (re.compile(r"splitk_reduce_kernel"), lambda m: "splitk"),
    (re.compile(r"attn_combine_kernel"), lambda m: "attn_combine"),
    (re.compile(r"attn_kernel"), lambda m: "attn"),
    (re.compile(r"gn_apply_kernel"), lambda m: "gn_apply"),
    (re.compile(r"gn_(partial|finalize)_kernel"), lambda m: "gn_stats"),
    (re.compile(r"layernorm_kernel"), lambda m: "layernorm"),
]
TAIR = re.compile(r"^(void )?(gemm_\w*kernel|conv_halo_kernel|splitk_reduce_kernel|gn_\w+|layernorm_kernel|attn_\w+|"
                  r"step_update_kernel|zero16_kernel|set_rows_kernel|advance_kernel)\b")


def key_of(name):
    for rx, f in KEY_RULES:
        m = rx.search(name)
        if m:
            return f(m)
    return "other"


def class_of(key):
    return key.split(":")[0] if ":" in key else key


def per_key(res, launches_csv, steps):
    """Traffic beyond L2 per denoise step (PMC, mean per dispatch x dispatches / steps) beside the algorithmic
    bytes of the launches of one profiled step (cldm.cpp's profile CSV: operands read once, outputs written
    once), per launch key and per kernel class; ratio = traffic / algorithmic."""
    alg = collections.defaultdict(float)
    tags = collections.defaultdict(set)
    for r in csv.DictReader(open(launches_csv)):
        alg[r["key"]] += float(r["alg_mb"]) * 1e6
        tags[r["key"]].add(r["tag"].split(" group=")[0])
    rows = collections.defaultdict(lambda: dict(traffic=0.0, dispatches=0.0, names=[]))
    for name, row in res.items():
        if not TAIR.match(name) or "hbm_read_bytes" not in row or "hbm_write_bytes" not in row:
            continue
        k = key_of(name)
        rows[k]["traffic"] += (row["hbm_read_bytes"] + row["hbm_write_bytes"]) * row["dispatches"] / steps
        rows[k]["dispatches"] += row["dispatches"] / steps
        rows[k]["names"].append(name)
    keys = {}
    for k in sorted(set(rows) | set(alg)):
        t = rows[k]["traffic"] if k in rows else 0.0
        a = alg.get(k, 0.0)
        keys[k] = dict(traffic_per_step=t, alg_per_step=a, ratio=(t / a) if a > 0 else None,
                       dispatches_per_step=rows[k]["dispatches"] if k in rows else 0.0,
                       kernels=rows[k]["names"] if k in rows else [], shapes=sorted(tags.get(k, [])))
    classes = collections.defaultdict(lambda: dict(traffic_per_step=0.0, alg_per_step=0.0, dispatches_per_step=0.0))
    for k, v in keys.items():
        c = classes[class_of(k)]
        for f in ("traffic_per_step", "alg_per_step", "dispatches_per_step"):
            c[f] += v[f]
    for c in classes.values():
        c["ratio"] = c["traffic_per_step"] / c["alg_per_step"] if c["alg_per_step"] > 0 else None
    return keys, dict(classes)


def main():
    args = sys.argv[1:]
    launches, steps = None, 3
    if "--launches" in args:
        i = args.index("--launches")
        launches = args[i + 1]
        del args[i:i + 2]
    if "--steps" in args:
        i = args.index("--steps")
        steps = int(args[i + 1])
        del args[i:i + 2]
    out, dirs = args[0], args[1:]
    per, names = load(dirs)
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for key, ctr in per.items():
        for c, v in ctr.items():
            agg[names[key]][c].append(v)
    res = {}
    for k, ctrs in agg.items():
        row = {"dispatches": max(len(v) for v in ctrs.values())}
        for c, vals in ctrs.items():
            row[c] = sum(vals) / len(vals)
        if "FETCH_SIZE" in row:
            row["hbm_read_bytes"] = 2 * 1024 * row["FETCH_SIZE"]
        if "WRITE_SIZE" in row:
            row["hbm_write_bytes"] = 1024 * row["WRITE_SIZE"]
        if "SQ_VALU_MFMA_BUSY_CYCLES" in row and row.get("GRBM_GUI_ACTIVE"):
            row["mfma_busy_frac"] = row["SQ_VALU_MFMA_BUSY_CYCLES"] / (row["GRBM_GUI_ACTIVE"] / N_XCD * N_SIMD)
        res[k] = row
    kernel_rows = dict(res)
    if launches:
        keys, classes = per_key(kernel_rows, launches, steps)
        res["_per_key"] = keys
        res["_per_class"] = classes
    # the build these counters measured: the source hash recorded beside the library the profiled process loaded
    # (bench.py reports this summary's traffic only while the hash equals the timed library's)
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from tair_amd import build as _build
    lib = _build.variant_lib(os.environ["TAIR_LIB_VARIANT"]) if os.environ.get("TAIR_LIB_VARIANT") else _build.LIB
    res["_src_hash"] = _build.library_hash(lib)
    json.dump(res, open(out, "w"), indent=1, sort_keys=True)
    print(f"source hash of the profiled library: {res['_src_hash']}")
    for k, row in sorted(kernel_rows.items(), key=lambda kv: -kv[1]["dispatches"]):
        extra = " ".join(f"{c}={row[c]:.4g}" for c in ("hbm_read_bytes", "hbm_write_bytes", "mfma_busy_frac")
                         if c in row)
        print(f"{row['dispatches']:6d} {k[:70]:70s} {extra}")
    if launches:
        print(f"\nper launch key, per denoise step (traffic = PMC bytes beyond L2; alg = operands read once, outputs "
              f"written once):")
        for k, v in sorted(keys.items(), key=lambda kv: -kv[1]["traffic_per_step"]):
            r = f"{v['ratio']:.2f}x" if v["ratio"] else "-"
            print(f"  {k:22s} {v['dispatches_per_step']:7.1f}/step  traffic {v['traffic_per_step'] / 1e9:8.3f} GB  "
                  f"alg {v['alg_per_step'] / 1e9:8.3f} GB  {r}")
        print("per class:")
        for k, v in sorted(classes.items(), key=lambda kv: -kv[1]["traffic_per_step"]):
            r = f"{v['ratio']:.2f}x" if v["ratio"] else "-"
            print(f"  {k:22s} {v['dispatches_per_step']:7.1f}/step  traffic {v['traffic_per_step'] / 1e9:8.3f} GB  "
                  f"alg {v['alg_per_step'] / 1e9:8.3f} GB  {r}")


if __name__ == "__main__":
    main()
