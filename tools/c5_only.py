"""Run only bench.py's C5 (1920x1080, 8k corners) leg and print its JSON (profiling helper).
usage: python tools/c5_only.py [chains groups] ..."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402

args = [int(a) for a in sys.argv[1:]] or [64, 1]
for i in range(0, len(args), 2):
    r = bench.c5_leg(torch.device("cuda"), chains=args[i], groups=args[i + 1])
    print(json.dumps({"chains": args[i], "groups": args[i + 1], "fps": r["frames_per_s"], "ms": r["ms_per_step"],
                      "ok": r["chains_ok"], "stages": r["stages_ms"]}), flush=True)
    torch.cuda.empty_cache()
