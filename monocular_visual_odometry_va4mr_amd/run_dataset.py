"""The reference driver (main.py) over a dataset folder, on the GPU pipeline.

    python -m monocular_visual_odometry_va4mr_amd.run_dataset --dataset kitti --path ./data/kitti \
        [--last-frame 2761] [--plot out/interface_plot.png] [--plot-every 0] [--poses out/poses.txt]

Same flow as main.py:
- dataset layout, K and ground-truth columns of utils.py:10-81 (KITTI sequence 05 image_0
  PNGs + poses/05.txt [-9,-1]; Malaga 800x600 rectified JPEGs, every second file from the
  third; Parking images/img_%05d.png + poses.txt);
- options, bootstrap pair and last frame of main.py:15-104 (options.py);
- VisualOdometryPipeLine(K, options).initialization(img0, img1), then continuous_operation
  for i in [bootstrap_frames[1] + 1, last_frame) (main.py:116-203);
- the interface figure (visualize.InterfacePlot) saved to out/interface_plot.png at the end,
  and every `--plot-every` frames if asked (main.py:201-205).

Frames are decoded one ahead of the pipeline on host threads (ingest.FrameSource) and copied
to HBM on their own stream; the timed loop covers continuous_operation only (the reference
times the whole script, main.py:10,207).  A synthetic sequence (no files) is available with
--dataset synthetic-kitti / synthetic-parking for a dry run.
"""
from __future__ import annotations

import argparse
import json
import os
import time

import numpy as np

from . import options as Op

K_KITTI = np.array([[7.188560000000e+02, 0, 6.071928000000e+02], [0, 7.188560000000e+02, 1.852157000000e+02], [0, 0, 1]])
K_MALAGA = np.array([[621.18428, 0, 404.0076], [0, 621.18428, 309.05989], [0, 0, 1]])
K_PARKING = np.array([[331.37, 0, 320], [0, 369.568, 240], [0, 0, 1]])
MALAGA_DIR = "malaga-urban-dataset-extract-07_rectified_800x600_Images"


def dataset_frames(dataset: str, path: str):
    """(K, frame paths, ground truth [n, 2] or empty) of utils.load_data_set / load_frame."""
    if dataset == "kitti":
        gt = np.loadtxt(os.path.join(path, "poses/05.txt"))[:, [-9, -1]]
        img_dir = os.path.join(path, "05/image_0")
        n = len([f for f in os.listdir(img_dir) if f.endswith(".png")])
        return K_KITTI, [os.path.join(img_dir, f"{i:06d}.png") for i in range(n)], gt
    if dataset == "malaga":
        d = os.path.join(path, MALAGA_DIR)
        left = sorted(os.listdir(d))[2::2]
        return K_MALAGA, [os.path.join(d, f) for f in left], np.zeros((0, 2))
    if dataset == "parking":
        gt = np.loadtxt(os.path.join(path, "poses.txt"))[:, [-9, -1]]
        img_dir = os.path.join(path, "images")
        n = len([f for f in os.listdir(img_dir) if f.startswith("img_")])
        return K_PARKING, [os.path.join(img_dir, f"img_{i:05d}.png") for i in range(n)], gt
    raise ValueError(f"unknown dataset {dataset!r}")


def run(dataset: str, path: str | None, last_frame: int | None = None, plot: str | None = "out/interface_plot.png",
        plot_every: int = 0, poses_out: str | None = None, device=None, verbose: bool = False, K=None) -> dict:
    """Run main.py's loop; returns a summary dict and (in "_vo") the pipeline object.
    K overrides the dataset's intrinsics (e.g. for a synthetic sequence written to disk)."""
    import torch

    from .VisualOdometryPipeLine import VisualOdometryPipeLine
    preset = dataset.replace("synthetic-", "")
    options, boot, ref_last = Op.get(preset)
    last = int(last_frame if last_frame is not None else ref_last)
    dev = torch.device(device or "cuda")
    if dataset.startswith("synthetic-"):
        from .synth import Renderer, poses
        rend = Renderer(preset, seed=1, device=dev)
        Rs, cs = poses(last, rend.p)
        K = rend.K
        gt = cs[:, [0, 2]]
        frames_iter = (rend.render_batch([i], Rs[i:i + 1], cs[i:i + 1])[0] for i in range(boot[1] + 1, last))
        img0 = rend.render_batch([boot[0]], Rs[boot[0]:boot[0] + 1], cs[boot[0]:boot[0] + 1])[0]
        img1 = rend.render_batch([boot[1]], Rs[boot[1]:boot[1] + 1], cs[boot[1]:boot[1] + 1])[0]
        src = None
    else:
        from . import ingest
        K_ds, paths, gt = dataset_frames(dataset, path)
        K = K_ds if K is None else np.asarray(K, np.float64)
        last = min(last, len(paths))
        img0 = ingest.imread_gray(paths[boot[0]])
        img1 = ingest.imread_gray(paths[boot[1]])
        h, w = img1.shape
        src = ingest.FrameSource([[p] for p in paths[boot[1] + 1:last]], w, h, device=dev)
        frames_iter = (f[0] for f in src)
    vo = VisualOdometryPipeLine(K, options, max_frames=last + 8, device=dev)
    vo.initialization(img0, img1)
    fig = None
    if plot:
        from .visualize import InterfacePlot
        fig = InterfacePlot(vo, img1, options, boot, gt)
    translations = [np.asarray(vo.transforms[-1][1], np.float64).reshape(3)]
    t_loop = 0.0
    n = 0
    try:
        for i, image in zip(range(boot[1] + 1, last), frames_iter):
            if verbose:
                print(f"\n\nProcessing frame {i}\n=====================")
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            vo.continuous_operation(image)
            torch.cuda.synchronize(dev)
            t_loop += time.perf_counter() - t0
            n += 1
            translations.append(np.asarray(vo.transforms[-1][1], np.float64).reshape(3))
            if fig is not None:
                fig.record(vo)
                if plot_every and (i - boot[1]) % plot_every == 0:
                    fig.update(vo, image, i)
                    fig.save(plot)
    finally:
        if src is not None:
            src.close()
    if fig is not None:
        fig.update(vo, image if n else img1, boot[1] + n)
        fig.save(plot)
        fig.close()
    tr = np.array(translations)
    if poses_out:
        from .evaluation import write_kitti_poses
        d = os.path.dirname(poses_out)
        if d:
            os.makedirs(d, exist_ok=True)
        write_kitti_poses(poses_out, vo.transforms)
    return {"dataset": dataset, "frames": n, "last_frame": last, "frames_per_s": round(n / max(t_loop, 1e-9), 1),
            "ms_per_frame": round(t_loop / max(n, 1) * 1e3, 3), "final_position": tr[-1].round(4).tolist(),
            "plot": plot, "poses": poses_out, "_vo": vo}


def main():
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--dataset", default="kitti",
                    choices=["kitti", "malaga", "parking", "synthetic-kitti", "synthetic-parking"])
    ap.add_argument("--path", default=None, help="dataset folder (utils.py:8-10 layout)")
    ap.add_argument("--last-frame", type=int, default=None)
    ap.add_argument("--plot", default="out/interface_plot.png", help="final interface PNG ('' to skip)")
    ap.add_argument("--plot-every", type=int, default=0, help="also redraw every N frames (0: final only)")
    ap.add_argument("--poses", default=None, help="write the trajectory as KITTI pose rows")
    ap.add_argument("--verbose", action="store_true")
    a = ap.parse_args()
    if not a.dataset.startswith("synthetic-") and not a.path:
        ap.error("--path is required for a dataset on disk")
    res = run(a.dataset, a.path, a.last_frame, a.plot or None, a.plot_every, a.poses, verbose=a.verbose)
    print(json.dumps({k: v for k, v in res.items() if not k.startswith("_")}))


if __name__ == "__main__":
    main()
