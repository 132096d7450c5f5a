import json, os, sys, time
sys.path.insert(0, "/root/repo")
import torch
import bench
from monocular_visual_odometry_va4mr_amd import options as Op
from monocular_visual_odometry_va4mr_amd.engine import Engine
from monocular_visual_odometry_va4mr_amd.synth import Renderer
mode = sys.argv[1]
dev = torch.device("cuda")
opts, (b0, b1), _ = Op.get("kitti")
gap = b1 - b0
rend = Renderer("kitti", seed=1, device=dev)
gt = bench.StagePoses(bench.SEQ_LEN, rend.p)
sample = bench.render_windows(rend, gt, [0], gap, 40, dev)[:, 0]
if mode in ("eager", "graph"):
    eng = Engine(rend.K, opts, rend.W, rend.H, batch=1, device=dev, ncap=16384, pcap=16384, fcap=64)
    eng.bootstrap(sample[0:1], sample[1:2])
    if mode == "graph":
        eng.capture_step()
        for i in range(2, sample.shape[0]):
            eng.step_graph(sample[i:i + 1]); eng.status_word(in_graph=True)
    else:
        for i in range(2, sample.shape[0]):
            eng.step(sample[i:i + 1]); eng.status_word()
    del eng
    torch.cuda.synchronize(); torch.cuda.empty_cache()
elif mode == "streams":
    ss = [torch.cuda.Stream(dev, priority=-1), torch.cuda.Stream(dev)]
    for s in ss:
        with torch.cuda.stream(s):
            torch.zeros(16, device=dev).add_(1)
    torch.cuda.synchronize()
seq = bench.sequence_leg(dev, 1, 0, 1, per_gpu=64)
print(json.dumps({"mode": mode, "seq": seq["frames_per_s"], "ok": seq["vs_reference"]["shards_identical"]}))
