#!/usr/bin/env python3
"""Per-(kernel, grid) launch statistics from a rocprofv3 --kernel-trace CSV: the stats summary
groups launches by name only, which mixes the headline workload with the bench's secondary
legs (single chain, C3, C5) whose launches of the same kernels have other grid sizes.

usage: trace_by_grid.py <prof_dir> <out.csv>"""
import csv
import glob
import re
import sys
from collections import defaultdict

f = glob.glob(f"{sys.argv[1]}/**/*kernel_trace.csv", recursive=True)[0]
acc = defaultdict(list)
for r in csv.DictReader(open(f)):
    m = re.search(r"(k_\w+(<[^>]*>)?)", r["Kernel_Name"])
    if not m:
        continue
    acc[(m.group(1), int(r["Grid_Size_X"]), int(r["Grid_Size_Y"]), int(r["Grid_Size_Z"]))].append(
        (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000)
with open(sys.argv[2], "w", newline="") as o:
    w = csv.writer(o)
    w.writerow(["kernel", "grid_x", "grid_y", "grid_z", "calls", "avg_us", "min_us", "max_us", "total_ms"])
    for k, v in sorted(acc.items(), key=lambda kv: -sum(kv[1])):
        w.writerow([k[0], k[1], k[2], k[3], len(v), round(sum(v) / len(v), 2), round(min(v), 2), round(max(v), 2),
                    round(sum(v) / 1e3, 3)])
