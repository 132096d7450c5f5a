"""Run only bench.py's C5 (1920x1080, 8k corners) leg and print its JSON (profiling helper)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402

print(json.dumps(bench.c5_leg(torch.device("cuda"))), flush=True)
