#!/usr/bin/env python
"""Critical-path view of one graph-replayed denoise step from a rocprofv3 kernel trace: wall time of
the step, summed kernel busy time per class, and idle gaps on the (merged) timeline."""
import csv
import re
import sys
from collections import defaultdict


def cls(name):
    for k, pat in [("halo", "conv_halo"), ("gemm", "gemm"), ("splitk", "splitk"), ("gn", "gn_"), ("ln", "layernorm"), ("attn", "attn"),
                   ("geglu", "geglu"), ("step", "step_update")]:
        if pat in name:
            return k
    return "other"


def main(path, step_marker="step_update", dump=None):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    marks = [i for i, r in enumerate(rows) if step_marker in r["Kernel_Name"]]
    print(f"{len(rows)} kernels, {len(marks)} step markers")
    if len(marks) < 3:
        return
    # take a step in the middle of the replayed run
    a, b = marks[len(marks) // 2], marks[len(marks) // 2 + 1]
    seg = rows[a + 1:b + 1]
    t0 = int(rows[a]["End_Timestamp"])
    t1 = int(rows[b]["End_Timestamp"])
    busy = defaultdict(float)
    cnt = defaultdict(int)
    ivs = []
    for r in seg:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        c = cls(r["Kernel_Name"])
        busy[c] += (e - s) / 1e3
        cnt[c] += 1
        ivs.append((s, e))
    ivs.sort()
    cover = 0
    cs, ce = ivs[0]
    for s, e in ivs[1:]:
        if s > ce:
            cover += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    cover += ce - cs
    wall = (t1 - t0) / 1e3
    print(f"step wall {wall:.1f} us, kernels {len(seg)}, union-busy {cover/1e3:.1f} us, idle {wall-cover/1e3:.1f} us")
    for k in sorted(busy, key=lambda k: -busy[k]):
        print(f"  {k:8s} n={cnt[k]:4d} sum={busy[k]:8.1f} us avg={busy[k]/cnt[k]:6.2f}")
    if dump:  # per-kernel timeline of the step: start offset, duration, gap to the previous end, grid, name
        with open(dump, "w") as f:
            prev_end = t0
            for r in seg:
                s_, e_ = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
                grid = "x".join(r.get(k, "?") for k in ("Grid_Size_X", "Grid_Size_Y", "Grid_Size_Z"))
                f.write(f"{(s_ - t0) / 1e3:9.2f} {(e_ - s_) / 1e3:8.2f} gap={(s_ - prev_end) / 1e3:7.2f} "
                        f"{grid:>16s} {r['Kernel_Name'][:90]}\n")
                prev_end = max(prev_end, e_)


if __name__ == "__main__":
    main(*sys.argv[1:])
