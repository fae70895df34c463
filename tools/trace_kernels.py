#!/usr/bin/env python
"""Per-launch listing of one replayed denoise step from a rocprofv3 kernel trace (name, grid, us)."""
import csv
import re
import sys


def short(n):
    n = re.sub(r"tair::\(anonymous namespace\)::", "", n)
    n = re.sub(r"\(.*", "", n)
    return n[:60]


rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
marks = [i for i, r in enumerate(rows) if "step_update" in r["Kernel_Name"]]
a, b = marks[len(marks) // 2], marks[len(marks) // 2 + 1]
prev_end = int(rows[a]["End_Timestamp"])
for r in rows[a + 1:b + 1]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    grid = f'{int(r["Grid_Size_X"])//int(r["Workgroup_Size_X"])}x{r["Grid_Size_Y"]}x{r["Grid_Size_Z"]}'
    print(f'{(e-s)/1e3:7.2f} gap={(s-prev_end)/1e3:5.2f} {short(r["Kernel_Name"]):55s} {grid} lds={r["LDS_Block_Size"]} vgpr={r["VGPR_Count"]}')
    prev_end = e
