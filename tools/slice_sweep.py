#!/usr/bin/env python3
"""Sequence-job plan sweep on one GPU: for each (world, shards per GPU,
overlap) the whole C2 sequence's plan is cut into world x B shards and rank 0's slice (B chains)
is run alone on this GPU, as one rank of a world-GPU job would (run_sequence.run without a
process group).  Prints one JSON line per configuration: the median wall of --reps runs (all
runs listed), bootstrap, steps, ms per step, the predicted job rate 4541 / wall, and the
per-shard comparison with the reference class's runs when a fixture holds that cut.

    python tools/slice_sweep.py W:B:O[:G] [W:B:O[:G] ...] [--reps 3]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from monocular_visual_odometry_va4mr_amd.run_sequence import reference_for, run  # noqa: E402


def main():
    argv = sys.argv[1:]
    reps = 3
    if "--reps" in argv:
        i = argv.index("--reps")
        reps = int(argv[i + 1])
        argv = argv[:i] + argv[i + 2:]
    dev = torch.device("cuda", 0)
    for spec in argv:
        parts = [int(v) for v in spec.split(":")]
        world, B, O = parts[:3]
        G = parts[3] if len(parts) > 3 else None         # stream groups (default: run_sequence's)
        ref = reference_for(os.path.join(ROOT, "tests", "golden"), world * B, O)
        runs = []
        for _ in range(reps):
            runs.append(run("kitti", 4541, B, overlap=O, seed=1, device=dev, rank=0, world=world, reference=ref,
                            time_boot=False, groups=G))
            torch.cuda.empty_cache()
        r = sorted(runs, key=lambda x: x["wall_s"])[len(runs) // 2]
        vs = r.get("vs_reference") or {}
        print(json.dumps({"world": world, "per_gpu": B, "overlap": O, "groups": r["groups"], "wall_s": r["wall_s"],
                          "wall_s_runs": [x["wall_s"] for x in runs], "bootstrap_s": r["bootstrap_s"],
                          "steps": r["steps"], "ms_per_step": round(r["step_s"] / max(1, r["steps"]) * 1e3, 4),
                          "host_launch_s": r["host_launch_s"],
                          "predicted_frames_per_s": round(4541 / r["wall_s"], 1), "shards_ok": r["shards_ok"],
                          "shards_compared": vs.get("shards_compared"), "shards_identical": vs.get("shards_identical")}),
              flush=True)


if __name__ == "__main__":
    main()
