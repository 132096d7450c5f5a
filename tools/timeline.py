#!/usr/bin/env python3
"""Per-queue kernel timeline of the last steps of a rocprofv3 --kernel-trace run: start/end
relative to the window start, and for each kernel the gap since the previous kernel on its
queue ended (time spent waiting for a dependency or for CUs).
usage: timeline.py <prof_dir> [n_last_kernels]"""
import csv
import glob
import re
import sys

f = glob.glob(f"{sys.argv[1]}/**/*kernel_trace.csv", recursive=True)[0]
rows = []
for r in csv.DictReader(open(f)):
    m = re.search(r"(k_\w+)", r["Kernel_Name"])
    name = m.group(1) if m else r["Kernel_Name"][:30]
    q = r.get("Queue_Id") or r.get("Stream_Id") or "?"
    rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), q, name, int(r["Grid_Size_X"])))
rows.sort()
n = int(sys.argv[2]) if len(sys.argv) > 2 else 160
rows = rows[-n:]
t0 = rows[0][0]
last_end = {}
print(f"{'start_us':>9} {'end_us':>9} {'dur_us':>8} {'gap_us':>8} queue kernel grid")
for s, e, q, name, g in rows:
    gap = (s - last_end[q]) / 1e3 if q in last_end else 0.0
    last_end[q] = e
    print(f"{(s - t0) / 1e3:9.1f} {(e - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f} {gap:8.1f} {q:>5} {name} {g}")
