#!/usr/bin/env python
"""Kernel statistics from a rocprofv3 --kernel-trace database (rocpd sqlite, ROCm 7.x).

    python tools/rocpd_stats.py RUN_results.db OUT_stats.csv [--step-kernel step_update_kernel]

Writes the classic `--stats` CSV (Name, Calls, TotalDurationNs, AverageNs, Percentage, MinNs, MaxNs)
and prints, per denoise step (delimited by the fused sampler kernel that ends each step), the
kernel count, the summed kernel time and the wall span first-start .. last-end of the step: span -
busy is the time the GPU spent between kernels (launch gaps / dependency bubbles), span < busy
means kernels overlapped (the ControlNet branch on its forked stream).
"""
from __future__ import annotations

import argparse
import collections
import csv
import sqlite3
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("out")
    ap.add_argument("--step-kernel", default="step_update_kernel")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute("select name, start, end from kernels order by start").fetchall()
    agg = collections.defaultdict(list)
    for name, s, e in rows:
        agg[name].append(e - s)
    tot = sum(sum(v) for v in agg.values())
    with open(a.out, "w", newline="") as f:
        w = csv.writer(f, quoting=csv.QUOTE_NONNUMERIC)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
        for name, d in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
            w.writerow([name, len(d), sum(d), sum(d) / len(d), 100.0 * sum(d) / tot, min(d), max(d)])
    # per-step spans: a step = the kernels after the previous step kernel up to this one
    steps, cur = [], []
    for name, s, e in rows:
        cur.append((s, e))
        if a.step_kernel in name:
            steps.append(cur)
            cur = []
    if steps:
        spans = [max(e for _, e in st) - min(s for s, _ in st) for st in steps[1:]]
        busy = [sum(e - s for s, e in st) for st in steps[1:]]
        n = [len(st) for st in steps[1:]]
        print(f"steps {len(steps)}: kernels/step median {statistics.median(n)}, busy/step median "
              f"{statistics.median(busy) / 1e3:.1f} us, span/step median {statistics.median(spans) / 1e3:.1f} us")
    for name, d in sorted(agg.items(), key=lambda kv: -sum(kv[1]))[:20]:
        print(f"{len(d):7d} {sum(d) / 1e6:9.2f} ms {sum(d) / len(d) / 1e3:8.2f} us {100 * sum(d) / tot:5.1f}%  {name[:100]}")


if __name__ == "__main__":
    main()
