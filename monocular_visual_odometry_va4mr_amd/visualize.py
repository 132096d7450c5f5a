"""Headless interface figure: the reference's 2x2 plot, rendered with
matplotlib's Agg backend into a PNG.

main.py:107-205 draws, after initialization and after every continuous_operation:
  [0,0] the current image with the PnP-RANSAC inliers (green x) and outliers (red x),
  [0,1] the full trajectory (t_x, t_z) with the ground truth (k--) when there is one,
  [1,0] the number of tracked landmarks over the last 20 frames,
  [1,1] the last 20 positions with the current landmarks (X, Z) in red,
with the axis limits main.py sets per frame (:184-198), and saves out/interface_plot.png
(:201-203).  `InterfacePlot` keeps the same artists and limits; it reads the attributes
main.py reads from the pipeline (transforms, num_pts, inlier_pts_current,
outlier_pts_current, matched_landmarks) from either the drop-in class or the reference's.
Drawing stays off the timed path: call update() only for the frames you want rendered
(the reference redraws every frame; `save_every` in run_dataset.py chooses how often).
"""
from __future__ import annotations

import os

import numpy as np


def _np(x, cols):
    a = np.asarray(x.cpu().numpy() if hasattr(x, "cpu") else x, dtype=np.float64)
    return a.reshape(-1, cols) if a.size else np.zeros((0, cols))


class InterfacePlot:
    def __init__(self, vo, image, options: dict, bootstrap_frames, ground_truth=None):
        import matplotlib
        matplotlib.use("Agg", force=True)
        import matplotlib.pyplot as plt
        self.plt = plt
        self.options = options
        self.boot = tuple(bootstrap_frames)
        gt = np.asarray(ground_truth if ground_truth is not None else [], dtype=np.float64)
        self.gt = gt.reshape(-1, 2) if gt.size else np.zeros((0, 2))
        # main.py:120-124
        t = np.asarray(vo.transforms[-1][1], dtype=np.float64)
        self.translations = t.reshape(-1, 3)
        self.num_tracked = np.array([vo.num_pts[-1]]).reshape(-1, 1)
        # main.py:107-108, 126-159
        self.fig, axs = plt.subplots(2, 2, figsize=(10, 8))
        self.axs = axs
        img = _img(image)
        outl = _np(vo.outlier_pts_current, 2)
        inl = _np(vo.inlier_pts_current, 2)
        self.image_plot = axs[0, 0].imshow(img, cmap="gray")
        self.outlier_plot = axs[0, 0].plot(outl[:, 0], outl[:, 1], "rx", markersize=6, label="Outliers")
        self.inlier_plot = axs[0, 0].plot(inl[:, 0], inl[:, 1], "gx", markersize=6, label="Inliers")
        axs[0, 0].set_title("Current image with RANSAC inliers and outliers")
        axs[0, 0].legend(loc=4, borderaxespad=0.)
        tr = self.translations
        self.trajectory_plot = axs[0, 1].plot(tr[:, 0], tr[:, 2], "bo-", linewidth=1, markersize=3, label="Trajectory")
        if len(self.gt) > 0:
            axs[0, 1].plot(self.gt[:, 0], self.gt[:, 1], "k--", label="Ground Truth")
        axs[0, 1].set_title("Full Trajectory")
        axs[0, 1].set_xlabel("X")
        axs[0, 1].set_ylabel("Y")
        axs[0, 1].legend(loc=4, borderaxespad=0.)
        self.num_plot = axs[1, 0].plot([0], self.num_tracked, "-", color="black", linewidth=1)
        axs[1, 0].set_title("# of tracked landmarks over the last 20 frames")
        axs[1, 0].set_xlabel("Frames")
        axs[1, 0].set_ylabel("# of Tracked Landmarks")
        self.trajectory_plot1 = axs[1, 1].plot(tr[:, 0], tr[:, 2], "bo-", linewidth=1, markersize=3, label="Trajectory")
        if len(self.gt) > 0:
            axs[1, 1].plot(self.gt[:, 0], self.gt[:, 1], "k--", label="Ground Truth")
        lm = _np(vo.matched_landmarks, 3)
        self.landmarks_plot = axs[1, 1].plot(lm[:, 0], lm[:, 2], "ro", markersize=6, label="Landmarks")
        axs[1, 1].set_title("Landmarks over the last 20 frames")
        axs[1, 1].set_xlabel("X")
        axs[1, 1].set_ylabel("Y")
        axs[1, 1].legend(loc=4, borderaxespad=0.)
        plt.tight_layout()

    def record(self, vo):
        """Per-frame bookkeeping of main.py:170-174 (cheap; no drawing)."""
        t = np.asarray(vo.transforms[-1][1], dtype=np.float64).reshape(1, 3)
        self.translations = np.append(self.translations, t, axis=0)
        self.num_tracked = np.append(self.num_tracked, vo.num_pts[-1])

    def update(self, vo, image, i: int):
        """Redraw for frame i (main.py:176-198); call record() for every frame first."""
        axs, tr, o = self.axs, self.translations, self.options
        self.image_plot.set_data(_img(image))
        outl = _np(vo.outlier_pts_current, 2)
        inl = _np(vo.inlier_pts_current, 2)
        if outl.shape[0] > 0:
            self.outlier_plot[0].set_data(outl[:, 0], outl[:, 1])
        self.inlier_plot[0].set_data(inl[:, 0], inl[:, 1])
        self.trajectory_plot[0].set_data(tr[:, 0], tr[:, 2])
        axs[0, 1].set_xlim([min(tr[:, 0]) - o["max_dist_landmarks"], max(tr[:, 0]) + o["max_dist_landmarks"]])
        axs[0, 1].set_ylim([min(tr[:, 2]) - o["max_dist_landmarks"], max(tr[:, 2]) + o["max_dist_landmarks"]])
        nt = self.num_tracked
        if i > self.boot[1] + 20:
            self.num_plot[0].set_data(np.arange(i - 19, i + 1), nt[-20:])
        else:
            self.num_plot[0].set_data(np.arange(self.boot[1], i + 1), nt)
        axs[1, 0].set_xlim([i - min(i, 21), i - 1])
        axs[1, 0].set_ylim([min(nt[max(-i, -20):]) - 10, max(nt[max(-i, -20):]) + 10])
        self.trajectory_plot1[0].set_data(tr[max(-i, -20):, 0], tr[max(-i, -20):, 2])
        lm = _np(vo.matched_landmarks, 3)
        self.landmarks_plot[0].set_data(lm[:, 0], lm[:, 2])
        axs[1, 1].set_xlim([tr[-1, 0] - o["max_dist_landmarks"], tr[-1, 0] + o["max_dist_landmarks"]])
        axs[1, 1].set_ylim([tr[-1, 2] - o["max_dist_landmarks"], tr[-1, 2] + o["max_dist_landmarks"]])

    def save(self, path: str = "out/interface_plot.png"):
        d = os.path.dirname(path)
        if d:
            os.makedirs(d, exist_ok=True)
        self.fig.savefig(path)
        return path

    def close(self):
        self.plt.close(self.fig)


def _img(image):
    a = image.cpu().numpy() if hasattr(image, "cpu") else np.asarray(image)
    return np.asarray(a, dtype=np.uint8)
