#!/usr/bin/env python3
"""Summarise rocprofv3 output for profiles/: per-kernel stats of this repo's kernels and,
from separate --pmc FETCH_SIZE / WRITE_SIZE passes, per-launch HBM bytes.

gfx950 correction (MI355X_MICROARCH.md "HBM"): FETCH_SIZE (KB) counts half the bytes of
wide coalesced reads -> x2; WRITE_SIZE (KB) is taken as is.

usage: prof_summary.py <tag> <prof_dir> [fetch_dir write_dir] [--chains B] [--steps N] [--groups G]
(--chains = chains per engine group, i.e. per launch)
(--steps N = warmup + timed steps of the profiled bench run: per-stage bytes are per step,
i.e. each kernel's mean bytes x its launches per step)
writes profiles/<tag>_kernel_stats.csv, profiles/<tag>_summary.md and (with PMC dirs)
profiles/traffic.json (read by bench.py for roofline.traffic)
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

STAGE_OF = {"k_lk": "track", "k_lk_w": "track", "k_eig": "gftt", "k_nms": "gftt", "k_eignms": "gftt", "k_gftt_select": "gftt",
            "k_ingest": "pyr_build", "k_pyrdown": "pyr_build", "k_pyr_level": "pyr_build", "k_pyr_rows": "pyr_build", "k_pyr_tail": "pyr_build", "k_scharr": "pyr_deriv",
            "k_pnp_ransac": "pnp", "k_pnp_apply": "pnp", "k_pnp_tri": "pnp", "k_pnp_fused": "pnp", "k_triangulate": "triangulate",
            "k_track_compact": "track", "k_add_finish": "add_finish", "k_eig3": "gftt", "k_lk_q": "track",
            "k_bf_prep": "match", "k_bf_mfma": "match", "k_bf_merge": "match", "k_bf_fixup": "match",
            "k_bf_prep_i8": "match", "k_bf_i8": "match", "k_add_finish_lean": "add_finish", "k_pyr01": "pyr_build",
            "k_gsel_gate": "gftt", "k_gsel_scan": "gftt", "k_gsel_scatter": "gftt", "k_gsel_rank": "gftt", "k_gsel_walk": "gftt"}


def short(name):
    n = name.split("(")[0] if not name.startswith("(") else name
    for tok in name.replace("(", " ").replace("<", " ").split():
        if "::k_" in tok:
            return tok.split("::")[-1]
        if tok.startswith("k_"):
            return tok
    return n[:40]


def pmc_avg(d, counter):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    acc = defaultdict(lambda: [0.0, 0])
    for f in files:
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") != counter:
                continue
            k = short(r["Kernel_Name"])
            acc[k][0] += float(r["Counter_Value"])
            acc[k][1] += 1
    return {k: v[0] / v[1] for k, v in acc.items() if v[1]}


def pmc_calls(d, counter):
    """launches per kernel in a --pmc pass (the per-step launch count comes from the PMC run,
    whose command may differ from the stats pass)"""
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    n = defaultdict(int)
    for f in files:
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") == counter:
                n[short(r["Kernel_Name"])] += 1
    return n


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    chains = None
    nsteps = None
    groups = 1
    if "--groups" in sys.argv:
        groups = int(sys.argv[sys.argv.index("--groups") + 1])
    if "--chains" in sys.argv:
        chains = int(sys.argv[sys.argv.index("--chains") + 1])
    if "--steps" in sys.argv:
        nsteps = int(sys.argv[sys.argv.index("--steps") + 1])
    flag_vals = {sys.argv[i + 1] for i, a in enumerate(sys.argv[:-1]) if a in ("--chains", "--steps", "--groups")}
    args = [a for a in args if a not in flag_vals]
    tag, prof = args[0], args[1]
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out_dir = os.path.join(root, "profiles")
    os.makedirs(out_dir, exist_ok=True)
    stats = glob.glob(os.path.join(prof, "**", "*kernel_stats.csv"), recursive=True)[0]
    rows = [r for r in csv.DictReader(open(stats)) if "at::" not in r["Name"]]
    with open(os.path.join(out_dir, f"{tag}_kernel_stats.csv"), "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=list(rows[0].keys()))
        w.writeheader()
        w.writerows(rows)
    fetch = write = {}
    ncalls = {}
    if len(args) >= 4:
        fetch, write = pmc_avg(args[2], "FETCH_SIZE"), pmc_avg(args[3], "WRITE_SIZE")
        ncalls = pmc_calls(args[2], "FETCH_SIZE")
    lines = [f"# rocprofv3 summary `{tag}`", "", "| kernel | calls | avg us | total ms | FETCH_SIZE x2 (MB/launch) | WRITE_SIZE (MB/launch) |",
             "|---|---:|---:|---:|---:|---:|"]
    traffic = {}
    for r in rows:
        k = short(r["Name"])
        fb = fetch.get(k)
        wb = write.get(k)
        fs = f"{2 * fb * 1024 / 1e6:.2f}" if fb is not None else "-"
        ws = f"{wb * 1024 / 1e6:.2f}" if wb is not None else "-"
        lines.append(f"| {k} | {r['Calls']} | {float(r['AverageNs']) / 1e3:.1f} | {float(r['TotalDurationNs']) / 1e6:.2f} | {fs} | {ws} |")
        if fb is not None and wb is not None and k in STAGE_OF:
            st = STAGE_OF[k]
            e = traffic.setdefault(st, {"bytes_per_launch": 0.0, "kernels": {}, "chains": chains,
                                        "groups": groups, "tag": tag})
            per_step = max(1, round(ncalls.get(k, 0) / (nsteps * groups))) if nsteps else 1
            b = (2 * fb * 1024 + wb * 1024) * per_step
            e["kernels"][k] = {"bytes_per_step": b, "launches_per_step": per_step}
            e["bytes_per_launch"] += b
    with open(os.path.join(out_dir, f"{tag}_summary.md"), "w") as f:
        f.write("\n".join(lines) + "\n")
    if traffic:
        with open(os.path.join(out_dir, "traffic.json"), "w") as f:
            json.dump(traffic, f, indent=1)
    print("\n".join(lines))


if __name__ == "__main__":
    main()
