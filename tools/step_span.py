#!/usr/bin/env python
"""Denoise-step duration from a rocprofv3 kernel trace: spacing of consecutive step_update_kernel
ends (one per hipGraph-replayed step), i.e. the profiler's view of what bench.py times with HIP events.

    python tools/step_span.py <kernel_trace.csv>
"""
import csv
import statistics
import sys

rows = [r for r in csv.DictReader(open(sys.argv[1])) if "step_update_kernel" in r["Kernel_Name"]]
ends = sorted(int(r["End_Timestamp"]) for r in rows)
d = [(b - a) / 1e6 for a, b in zip(ends, ends[1:])]
d = [x for x in d if x < 50.0]  # drop the gaps between restorations (VAE decode, host work)
print(f"step_update launches {len(ends)}; steady step spacing: median {statistics.median(d):.4f} ms, "
      f"mean {statistics.mean(d):.4f} ms over {len(d)} steps")
