#!/usr/bin/env python3
"""Phase times of k_gftt_select (block 0 of the launch) on the headline workload: B KITTI
chains, every stage on one stream.  Needs the diagnostics build
(make -C monocular_visual_odometry_va4mr_amd/csrc ../_build/libvo_hip_selprof.so).
usage: python tools/sel_prof.py [B] [steps] [preset]"""
import ctypes as C
import os
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["VO_HIP_LIB"] = os.path.join(HERE, "monocular_visual_odometry_va4mr_amd", "_build", "libvo_hip_selprof.so")
os.environ["VO_ONE_STREAM"] = "1"
sys.path.insert(0, HERE)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from monocular_visual_odometry_va4mr_amd import _lib as L  # noqa: E402
from monocular_visual_odometry_va4mr_amd import options as Op  # noqa: E402
from monocular_visual_odometry_va4mr_amd.engine import Engine  # noqa: E402
from monocular_visual_odometry_va4mr_amd.synth import Renderer, poses  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 384
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 6
preset = sys.argv[3] if len(sys.argv) > 3 else "kitti"
dev = torch.device("cuda")
r = Renderer(preset, seed=1, device=dev)
opts, (b0, b1), n_seq = Op.get(preset)
n = steps + b1 + 2
Rs, cs = poses(n_seq, r.p)
starts = [(i * (n_seq - n)) // max(1, B) for i in range(B)]
frames = torch.stack([r.render_batch(list(range(s, s + n)), Rs[s:s + n], cs[s:s + n]) for s in starts], 1)
cap = 65536 if preset == "hd1080" else 16384
eng = Engine(r.K, opts, r.W, r.H, batch=B, device=dev, ncap=cap, pcap=cap, fcap=n + 8)
eng.bootstrap(frames[b0], frames[b1])
lib = L.lib()
lib.vo_select_prof_read.argtypes = [C.c_void_p]
buf = (C.c_longlong * 16)()
for i in range(b1 + 1, n):
    eng.step(frames[i])
    torch.cuda.synchronize()
    lib.vo_select_prof_read(buf)
    t = np.array(buf[:16], dtype=np.int64)
    us = lambda a, b: (t[b] - t[a]) / 100.0  # noqa: E731  (100 MHz)
    print(f"step {i}: gate+compact {us(0, 1):7.1f} | page gather {us(1, 2):7.1f} | sort {us(2, 3):7.1f} | "
          f"conflicts {us(3, 5):7.1f} | rounds {us(5, 6):7.1f} ({t[10]}) | emit {us(6, 4):7.1f} | total {us(0, 4):7.1f} us"
          f" | passing {int(eng.t['gf_n'][0])} corners {int(eng.t['nCorners'][0])}", flush=True)
