#!/usr/bin/env python3
"""Per-kernel mean of every counter in rocprofv3 --pmc output dirs (tools/gpu_sq.sh).
usage: sq_summary.py <dir> [<dir> ...]"""
import csv, glob, sys
from collections import defaultdict

acc = defaultdict(lambda: defaultdict(lambda: [0.0, 0]))
for d in sys.argv[1:]:
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            n = r["Kernel_Name"]
            k = next((t.split("::")[-1] for t in n.replace("(", " ").replace("<", " ").split() if "::k_" in t), n[:30])
            a = acc[k][r["Counter_Name"]]
            a[0] += float(r["Counter_Value"]); a[1] += 1
for k, cs in acc.items():
    m = {c: v[0] / v[1] for c, v in cs.items()}
    print(k)
    for c in sorted(m):
        print(f"   {c:24s} {m[c]:16.0f}")
    w = m.get("SQ_WAVES")
    if w:
        for c in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD"):
            if c in m:
                print(f"   {c + '/wave':24s} {m[c] / w:16.1f}")
        if "SQ_WAVE_CYCLES" in m:
            for c in ("SQ_WAIT_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_VALU"):
                if c in m:
                    print(f"   {c + '/wavecyc':24s} {m[c] / m['SQ_WAVE_CYCLES']:16.3f}")
