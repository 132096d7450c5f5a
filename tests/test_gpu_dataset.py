"""main.py's driver over a dataset folder (run_dataset.py): files -> ingest -> drop-in class ->
trajectory + interface PNG; the trajectory equals the golden reference run on the same frames."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")
PIL = pytest.importorskip("PIL.Image")


def test_parking_folder_run_matches_golden(tmp_path):
    from conftest import golden_frames, load_golden
    from monocular_visual_odometry_va4mr_amd import ingest
    from monocular_visual_odometry_va4mr_amd import run_dataset as R
    g = load_golden("parking_c1")
    fr = golden_frames(g)[:20]
    (tmp_path / "images").mkdir()
    for i, f in enumerate(fr):
        PIL.fromarray(f, mode="L").save(tmp_path / "images" / f"img_{i:05d}.png")
    np.savetxt(tmp_path / "poses.txt", np.zeros((len(fr), 12)))
    png = str(tmp_path / "out" / "interface_plot.png")
    res = R.run("parking", str(tmp_path), last_frame=len(fr), plot=png, plot_every=5,
                poses_out=str(tmp_path / "out" / "poses.txt"), K=g["K"])
    vo = res["_vo"]
    t = np.array([np.asarray(x).ravel() for _, x in vo.transforms[1:]])
    assert res["frames"] == len(fr) - 7
    assert np.array_equal(t, g["t"][:len(t), :, 0])
    assert np.array_equal(np.asarray(vo.num_pts), g["num_pts"][:len(vo.num_pts)])
    w, h, _, _ = ingest.png_info(open(png, "rb").read())
    assert (w, h) == (1000, 800)
    rows = np.loadtxt(tmp_path / "out" / "poses.txt")
    assert rows.shape == (len(vo.transforms), 12)


def test_synthetic_dry_run():
    from monocular_visual_odometry_va4mr_amd import run_dataset as R
    res = R.run("synthetic-kitti", None, last_frame=12, plot=None)
    assert res["frames"] == 12 - 3 and res["frames_per_s"] > 0
