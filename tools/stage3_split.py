#!/usr/bin/env python
"""Split each step of the configs[4] prompt loop (between consecutive step_update_kernel launches of
a rocprofv3 kernel trace) into the HIP denoise-step kernels (tair::) and everything else (the
stock-torch TESTR / CLIP-H towers, copies), by busy time and by the step's wall time."""
import csv
import sys
from collections import defaultdict


def main(path):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    marks = [i for i, r in enumerate(rows) if "step_update" in r["Kernel_Name"]]
    print(f"{len(rows)} kernels, {len(marks)} step markers")
    walls, tair_busy, other_busy = [], [], []
    top = defaultdict(float)
    for a, b in zip(marks[len(marks) // 2:-1], marks[len(marks) // 2 + 1:]):
        seg = rows[a + 1:b + 1]
        walls.append((int(rows[b]["End_Timestamp"]) - int(rows[a]["End_Timestamp"])) / 1e3)
        tb = ob = 0.0
        for r in seg:
            d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            if "tair::" in r["Kernel_Name"] or "msda" in r["Kernel_Name"]:
                tb += d
            else:
                ob += d
                top[r["Kernel_Name"][:90]] += d
        tair_busy.append(tb)
        other_busy.append(ob)
    n = len(walls)
    print(f"steps {n}: wall {sum(walls) / n:.1f} us, tair kernels busy {sum(tair_busy) / n:.1f} us, "
          f"other kernels busy {sum(other_busy) / n:.1f} us")
    for k, v in sorted(top.items(), key=lambda kv: -kv[1])[:15]:
        print(f"  {v / n:8.1f} us/step  {k}")


if __name__ == "__main__":
    main(sys.argv[1])
