"""Headless interface figure (main.py:107-205) and the dataset-folder driver's loaders (CPU)."""
import os

import numpy as np
import pytest

pytest.importorskip("matplotlib")


class _FakeVO:
    """The attributes main.py reads from the pipeline."""

    def __init__(self, rng, k):
        self.transforms = [(np.eye(3), np.array([[0.1 * j], [0.0], [1.0 * j]])) for j in range(k + 1)]
        self.num_pts = [100 + j for j in range(k + 1)]
        self.inlier_pts_current = rng.uniform(0, 300, (50, 2)).astype(np.float32)
        self.outlier_pts_current = rng.uniform(0, 300, (7, 2)).astype(np.float32)
        self.matched_landmarks = rng.uniform(-20, 20, (60, 3)).astype(np.float32)


def test_interface_plot_png(tmp_path):
    from monocular_visual_odometry_va4mr_amd import ingest, options
    from monocular_visual_odometry_va4mr_amd.visualize import InterfacePlot
    rng = np.random.default_rng(0)
    opts, boot, _ = options.get("parking")
    img = rng.integers(0, 256, (240, 320), dtype=np.uint8)
    vo = _FakeVO(rng, 0)
    gt = np.c_[np.linspace(0, 3, 40), np.linspace(0, 30, 40)]
    fig = InterfacePlot(vo, img, opts, boot, gt)
    for i in range(boot[1] + 1, boot[1] + 30):                      # > 20 frames: sliding window
        vo = _FakeVO(rng, i - boot[1])
        fig.record(vo)
    fig.update(vo, img, boot[1] + 29)
    out = fig.save(str(tmp_path / "out" / "interface_plot.png"))
    fig.close()
    assert len(fig.translations) == 30 and len(fig.num_tracked) == 30
    w, h, _, _ = ingest.png_info(open(out, "rb").read())
    assert (w, h) == (1000, 800)                                    # figsize (10, 8) at 100 dpi
    xl = fig.axs[1, 1].get_xlim()
    assert np.isclose(xl[0], fig.translations[-1, 0] - opts["max_dist_landmarks"])


def test_dataset_layouts(tmp_path):
    """utils.py:10-81 folder layouts, K and ground-truth columns [-9, -1]."""
    from monocular_visual_odometry_va4mr_amd import run_dataset as R
    kitti = tmp_path / "kitti"
    (kitti / "05" / "image_0").mkdir(parents=True)
    (kitti / "poses").mkdir()
    for i in range(3):
        (kitti / "05" / "image_0" / f"{i:06d}.png").write_bytes(b"")
    rows = np.arange(3 * 12, dtype=np.float64).reshape(3, 12)
    np.savetxt(kitti / "poses" / "05.txt", rows)
    K, paths, gt = R.dataset_frames("kitti", str(kitti))
    assert np.allclose(K, R.K_KITTI) and len(paths) == 3 and paths[2].endswith("05/image_0/000002.png")
    assert np.array_equal(gt, rows[:, [3, 11]])
    mal = tmp_path / "malaga" / R.MALAGA_DIR
    mal.mkdir(parents=True)
    for i in range(8):
        (mal / f"img_{i:02d}_{'left' if i % 2 == 0 else 'right'}.jpg").write_bytes(b"")
    K, paths, gt = R.dataset_frames("malaga", str(tmp_path / "malaga"))
    names = sorted(os.listdir(mal))[2::2]
    assert [os.path.basename(p) for p in paths] == names and len(gt) == 0
    park = tmp_path / "parking"
    (park / "images").mkdir(parents=True)
    for i in range(4):
        (park / "images" / f"img_{i:05d}.png").write_bytes(b"")
    np.savetxt(park / "poses.txt", rows)
    K, paths, gt = R.dataset_frames("parking", str(park))
    assert np.allclose(K, R.K_PARKING) and len(paths) == 4 and gt.shape == (3, 2)
