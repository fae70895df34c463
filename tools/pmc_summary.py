#!/usr/bin/env python
"""Per-kernel PMC summary from rocprofv3 `--pmc ... --output-format csv` counter files.

    python tools/pmc_summary.py OUT.json DIR [DIR ...]

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


def main():
    out, dirs = sys.argv[1], sys.argv[2:]
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
    json.dump(res, open(out, "w"), indent=1, sort_keys=True)
    for k, row in sorted(res.items(), key=lambda kv: -kv[1]["dispatches"]):
        extra = " ".join(f"{c}={row[c]:.4g}" for c in ("hbm_read_bytes", "hbm_write_bytes", "mfma_busy_frac")
                         if c in row)
        print(f"{row['dispatches']:6d} {k[:70]:70s} {extra}")


if __name__ == "__main__":
    main()
