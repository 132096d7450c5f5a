#!/usr/bin/env python3
"""Per-pyramid-level view of the k_lk dispatches in rocprofv3 CSV output.

k_lk is launched once per level, coarse to fine, every step, so the i-th dispatch of a
run is level L - (i mod (L+1)).  usage: lk_levels.py <dir> [--levels 5]
Prints mean duration (kernel_trace) and mean counter values (counter_collection) by level.
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def main():
    d = sys.argv[1]
    nl = int(sys.argv[sys.argv.index("--levels") + 1]) if "--levels" in sys.argv else 5
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        rows = [r for r in csv.DictReader(open(f)) if "k_lk" in r["Kernel_Name"]]
        rows.sort(key=lambda r: int(r["Start_Timestamp"]))
        acc = defaultdict(list)
        for i, r in enumerate(rows):
            acc[nl - 1 - i % nl].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
        for lv in sorted(acc):
            v = acc[lv]
            print(f"level {lv}: {len(v)} launches, mean {sum(v) / len(v):.1f} us")
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        rows = [r for r in csv.DictReader(open(f)) if "k_lk" in r["Kernel_Name"]]
        disp = sorted({int(r["Dispatch_Id"]) for r in rows})
        lvl = {dd: nl - 1 - i % nl for i, dd in enumerate(disp)}
        acc = defaultdict(lambda: defaultdict(list))
        for r in rows:
            acc[lvl[int(r["Dispatch_Id"])]][r["Counter_Name"]].append(float(r["Counter_Value"]))
        for lv in sorted(acc):
            print(f"level {lv}: " + ", ".join(f"{c}={sum(v) / len(v):.3g}" for c, v in sorted(acc[lv].items())))


if __name__ == "__main__":
    main()
