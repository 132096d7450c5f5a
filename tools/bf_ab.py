"""A/B of the BF 2-NN kernels on the C5 / C3 match legs: int8 default vs VO_BF_BF16=1, and
the libraries named in argv (VO_HIP_LIB variants) in subprocesses."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def leg():
    import torch
    sys.path.insert(0, ROOT)
    import bench
    dev = torch.device("cuda")
    c5 = bench.c5_sift_leg(dev, iters=5)
    c3 = bench.c3_leg(dev, iters=5)
    return {"c5_bf_ms_per_pair": c5["bf_ms_per_pair"], "c5_tops": c5["bf_roofline"]["achieved"],
            "c3_bf_ms_per_pair": c3["bf_ms_per_pair"], "c3_tops": c3["bf_roofline"]["achieved"]}


if len(sys.argv) > 1 and sys.argv[1] == "--leg":
    print("RESULT " + json.dumps(leg()), flush=True)
    sys.exit(0)

runs = [("i8", {}), ("bf16", {"VO_BF_BF16": "1"})] + [(os.path.basename(p), {"VO_HIP_LIB": os.path.abspath(p)})
                                                       for p in sys.argv[1:]]
for name, env in runs:
    e = dict(os.environ)
    e.update(env)
    r = subprocess.run([sys.executable, os.path.abspath(__file__), "--leg"], env=e, capture_output=True, text=True,
                       timeout=240)
    res = [l for l in r.stdout.splitlines() if l.startswith("RESULT ")]
    print(name, res[0][7:] if res else ("FAILED rc=%d %s" % (r.returncode, r.stderr[-500:])), flush=True)
    if not res:
        sys.exit(1)
