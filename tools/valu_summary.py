#!/usr/bin/env python3
"""VALU roofline input for bench.py: per-launch SQ instruction counts of k_lk_w from the
--pmc passes of tools/gpu_sq.sh, divided by the points that launch tracked.

usage: valu_summary.py <sq1_dir> <sq2_dir> <bench_json_of_the_same_run> <out.json> [tag]
The bench JSON (same --chains/--groups/--steps as the SQ passes) gives the points tracked per
launch (points_last_step: landmarks + candidates of the group's chains).  bench.py then
reports achieved VALU wave-instructions/s = valu_per_point x live points / live track time
against the issue peak (CDNA4: 32-wide SIMDs, a wave64 VALU instruction issues in 2 cycles;
1024 SIMDs x 2.4 GHz / 2 = 1.2288e12 wave-instructions/s)."""
import csv
import glob
import json
import sys
from collections import defaultdict


def counters(dirs):
    acc = defaultdict(lambda: defaultdict(lambda: [0.0, 0]))
    for d in dirs:
        for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                if "k_lk_w" not in r["Kernel_Name"]:
                    continue
                a = acc["k_lk_w"][r["Counter_Name"]]
                a[0] += float(r["Counter_Value"])
                a[1] += 1
    return {k: {c: v[0] / v[1] for c, v in cs.items()} for k, cs in acc.items()}


def main():
    sq1, sq2, bj, out = sys.argv[1:5]
    tag = sys.argv[5] if len(sys.argv) > 5 else ""
    m = counters([sq1, sq2])["k_lk_w"]
    b = json.load(open(bj))
    pts = float(b["points_last_step"])
    # one k_lk_w launch tracks one stream group's chains (points_last_step counts group 0's)
    per_launch = b["config"]["chains_per_gpu"] // max(1, int(b["config"].get("streams_per_gpu", 1)))
    rec = {"kernel": "k_lk_w", "tag": tag, "chains_per_launch": per_launch, "points_per_launch": pts,
           "valu_insts_per_launch": m["SQ_INSTS_VALU"], "salu_insts_per_launch": m.get("SQ_INSTS_SALU"),
           "lds_insts_per_launch": m.get("SQ_INSTS_LDS"), "waves_per_launch": m.get("SQ_WAVES"),
           "valu_per_point": m["SQ_INSTS_VALU"] / pts,
           "wait_inst_any_per_wave_cycle": m.get("SQ_WAIT_INST_ANY", 0) / m["SQ_WAVE_CYCLES"] if "SQ_WAVE_CYCLES" in m else None,
           "active_valu_per_wave_cycle": m.get("SQ_ACTIVE_INST_VALU", 0) / m["SQ_WAVE_CYCLES"] if "SQ_WAVE_CYCLES" in m else None,
           "lds_bank_conflict_per_lds_inst": m.get("SQ_LDS_BANK_CONFLICT", 0) / max(1.0, m.get("SQ_INSTS_LDS", 1.0))}
    json.dump(rec, open(out, "w"), indent=1)
    print(json.dumps(rec))


if __name__ == "__main__":
    main()
