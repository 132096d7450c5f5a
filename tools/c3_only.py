"""Run only bench.py's C3 (1024x768 SIFT + batched BF) and C5 SIFT/BF legs and print their JSON
(A/B helper).  usage: python tools/c3_only.py [reps]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402

dev = torch.device("cuda")
for _ in range(int(sys.argv[1]) if len(sys.argv) > 1 else 1):
    r = bench.c3_leg(dev)
    r5 = bench.c5_sift_leg(dev)
    print(json.dumps({"c3_bf_ms_per_pair": r["bf_ms_per_pair"], "c3_pairs_per_s": r["pairs_per_s"],
                      "c3_bf_frac": (r.get("bf_roofline") or {}).get("frac"),
                      "c5_bf_ms_per_pair": r5["bf_ms_per_pair"], "c5_bf_frac": (r5.get("bf_roofline") or {}).get("frac")}),
          flush=True)
    torch.cuda.empty_cache()
