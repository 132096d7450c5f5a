#!/usr/bin/env python3
"""Average SQ counters per (kernel, grid) from rocprofv3 --pmc output directories.
usage: sq_table.py <dir> [<dir> ...] [--kernel SUBSTR]"""
import csv
import glob
import sys
from collections import defaultdict

dirs = [a for a in sys.argv[1:] if not a.startswith("--")]
ksub = sys.argv[sys.argv.index("--kernel") + 1] if "--kernel" in sys.argv else ""
acc = defaultdict(lambda: defaultdict(list))
for d in dirs:
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"].split("(")[1] if r["Kernel_Name"].startswith("(anon") else r["Kernel_Name"]
            name = name.split("::")[-1] if "::" in name else name
            if ksub and ksub not in r["Kernel_Name"]:
                continue
            acc[(name[:24], r.get("Grid_Size", "?"))][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in sorted(acc.items()):
    print(k[0], "grid", k[1])
    for c, v in sorted(cs.items()):
        print(f"   {c:24s} {sum(v) / len(v):16.4g}")
