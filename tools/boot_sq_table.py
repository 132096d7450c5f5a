"""Per-kernel issue balance of tools/boot_trace.sh's --pmc pass over the 768-chain bootstrap
(boot_prof.py, three calls): busy time per launch, VALU / SALU share of issue, instruction totals.
usage: boot_sq_table.py <counter_collection.csv> [<before.csv>]"""
import csv
import re
import sys
from collections import defaultdict


def load(path):
    acc = defaultdict(lambda: defaultdict(float))
    n = defaultdict(int)
    for r in csv.DictReader(open(path)):
        m = re.search(r"(k_\w+(<\d+>)?)", r["Kernel_Name"])
        k = m.group(1) if m else r["Kernel_Name"][:30]
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
        if r["Counter_Name"] == "SQ_BUSY_CU_CYCLES":
            n[k] += 1
    return acc, n


acc, n = load(sys.argv[1])
before = load(sys.argv[2])[0] if len(sys.argv) > 2 else {}
for k, c in sorted(acc.items(), key=lambda kv: -kv[1].get("SQ_BUSY_CU_CYCLES", 0)):
    b = c["SQ_BUSY_CU_CYCLES"]
    line = (f"{k:20s} launches {n[k]:4d} busy/launch {b / 256 / 2.4e3 / n[k]:8.1f} us  SALU {c['SQ_INST_CYCLES_SALU'] / b:.2f}"
            f"  VALU {c['SQ_INSTS_VALU'] * 2 / 4 / b:.2f}  VALU {c['SQ_INSTS_VALU']:.3g}  SALU {c['SQ_INSTS_SALU']:.3g}")
    if k in before:
        line += (f"  | before: busy {before[k]['SQ_BUSY_CU_CYCLES'] / 256 / 2.4e3 / n[k]:8.1f} us  VALU {before[k]['SQ_INSTS_VALU']:.3g}"
                 f"  SALU {before[k]['SQ_INSTS_SALU']:.3g}")
    print(line)
