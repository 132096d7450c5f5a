"""Frame ingest: PNG decode (libvo_ingest.so) vs PIL and the libpng gray formula (CPU)."""
import os

import numpy as np
import pytest

PIL = pytest.importorskip("PIL.Image")


def _gray_ref(rgb):
    """libpng 1.6 png_set_rgb_to_gray(1, 0.299, 0.587) without gamma (OpenCV's IMREAD_GRAYSCALE
    path for colour PNGs): truncated 15-bit weights 9797 / 19234 / 3737, truncating shift,
    gray pixels passed through (parity with libpng itself unpinned: it is not in this image)."""
    rgb = rgb.astype(np.int64)
    rc, gc = (29900 * 32768) // 100000, (58700 * 32768) // 100000
    bc = 32768 - rc - gc
    g = (rc * rgb[..., 0] + gc * rgb[..., 1] + bc * rgb[..., 2]) >> 15
    same = (rgb[..., 0] == rgb[..., 1]) & (rgb[..., 0] == rgb[..., 2])
    return np.where(same, rgb[..., 0], g).astype(np.uint8)


@pytest.fixture(scope="module")
def frames():
    from monocular_visual_odometry_va4mr_amd.synth import make_sequence
    fr, _, _, _ = make_sequence("parking", 3, seed=5)
    return fr


def test_png_gray_roundtrip_exact(tmp_path, frames):
    from monocular_visual_odometry_va4mr_amd import ingest
    for i, f in enumerate(frames):
        p = tmp_path / f"img_{i:05d}.png"
        PIL.fromarray(f, mode="L").save(p, optimize=(i % 2 == 0))     # different filter choices
        g = ingest.imread_gray(str(p))
        assert np.array_equal(g, f)


def test_png_color_and_16bit_to_gray(tmp_path, frames):
    from monocular_visual_odometry_va4mr_amd import ingest
    rng = np.random.default_rng(0)
    rgb = np.stack([frames[0], frames[1], frames[2]], -1)
    p = tmp_path / "rgb.png"
    PIL.fromarray(rgb, mode="RGB").save(p)
    assert np.array_equal(ingest.imread_gray(str(p)), _gray_ref(rgb))
    rgba = np.concatenate([rgb, rng.integers(0, 256, rgb.shape[:2] + (1,), dtype=np.uint8)], -1)
    p = tmp_path / "rgba.png"
    PIL.fromarray(rgba, mode="RGBA").save(p)
    assert np.array_equal(ingest.imread_gray(str(p)), _gray_ref(rgb))
    pal = PIL.fromarray(rgb[:64, :64], mode="RGB").quantize(colors=32)
    p = tmp_path / "pal.png"
    pal.save(p)
    exp = _gray_ref(np.asarray(pal.convert("RGB")))
    assert np.array_equal(ingest.imread_gray(str(p)), exp)
    g16 = (frames[0].astype(np.uint16) << 8) | 0x5A
    p = tmp_path / "g16.png"
    PIL.fromarray(g16.astype(np.int32), mode="I").convert("I;16").save(p)
    assert np.array_equal(ingest.imread_gray(str(p)), frames[0])


def test_bad_inputs_fail_loudly(tmp_path):
    from monocular_visual_odometry_va4mr_amd import ingest
    p = tmp_path / "x.png"
    p.write_bytes(b"not a png")
    with pytest.raises(ValueError):
        ingest.imread_gray(str(p))


def test_frame_source_cpu_batches_in_order(tmp_path, frames):
    from monocular_visual_odometry_va4mr_amd import ingest
    paths = []
    for i in range(6):
        p = tmp_path / f"f{i}.png"
        PIL.fromarray(np.roll(frames[i % 3], i, axis=1), mode="L").save(p)
        paths.append(str(p))
    batches = [[paths[j], paths[(j + 3) % 6]] for j in range(5)]
    src = ingest.FrameSource(batches, frames.shape[2], frames.shape[1], device="cpu", threads=4)
    got = [t.numpy().copy() for t in src]
    src.close()
    assert len(got) == 5
    for j, g in enumerate(got):
        assert np.array_equal(g[0], np.roll(frames[j % 3], j, axis=1))
        assert np.array_equal(g[1], np.roll(frames[((j + 3) % 6) % 3], (j + 3) % 6, axis=1))
    # a missing file is reported, not skipped
    src = ingest.FrameSource([[paths[0], str(tmp_path / "missing.png")]], frames.shape[2], frames.shape[1],
                             device="cpu")
    with pytest.raises(RuntimeError):
        list(src)
    src.close()


def test_ingest_header_symbols_exported():
    import subprocess
    from monocular_visual_odometry_va4mr_amd import ingest
    ingest.lib()
    out = subprocess.run(["nm", "-D", "--defined-only", ingest.INGEST_PATH], capture_output=True, text=True).stdout
    defined = {ln.split()[-1] for ln in out.splitlines() if ln.strip()}
    hdr = open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include", "vo_ingest.h")).read()
    import re
    declared = set(re.findall(r"\b(vo_[a-z0-9_]+)\s*\(", hdr))
    assert declared and declared <= defined, declared - defined


def test_jpeg_gray_matches_decoder_luma(tmp_path, frames):
    """Malaga JPEGs: grayscale straight from the decoder (the Y plane), like OpenCV's
    IMREAD_GRAYSCALE JPEG path; a gray JPEG decodes to PIL's own result exactly."""
    from monocular_visual_odometry_va4mr_amd import ingest
    p = tmp_path / "g.jpg"
    PIL.fromarray(frames[0], mode="L").save(p, quality=95)
    g = ingest.imread_gray(str(p))
    assert g.dtype == np.uint8 and g.shape == frames[0].shape
    assert np.array_equal(g, np.asarray(PIL.open(p)))
    assert np.abs(g.astype(int) - frames[0]).mean() < 3.0            # lossy but close
    rgb = np.stack([frames[0], frames[1], frames[2]], -1)
    p = tmp_path / "c.jpg"
    PIL.fromarray(rgb, mode="RGB").save(p, quality=95)
    y = ingest.imread_gray(str(p))
    ycc = np.asarray(PIL.open(p).convert("YCbCr"))[..., 0]            # luma via RGB round trip
    assert y.shape == rgb.shape[:2] and np.abs(y.astype(int) - ycc).max() <= 3
    assert ingest.is_jpeg(str(p))


def test_frame_source_jpeg_and_mixed_batches(tmp_path, frames):
    from monocular_visual_odometry_va4mr_amd import ingest
    paths = []
    for i, f in enumerate(frames):
        p = tmp_path / (f"f{i}.jpg" if i % 2 == 0 else f"f{i}.png")
        PIL.fromarray(f, mode="L").save(p, **({"quality": 97} if i % 2 == 0 else {}))
        paths.append(str(p))
    h, w = frames[0].shape
    src = ingest.FrameSource([paths[:2], paths[2:3] + paths[:1]], w, h, device="cpu", threads=2)
    out = [b.clone() for b in src]
    src.close()
    assert len(out) == 2 and tuple(out[0].shape) == (2, h, w)
    assert np.array_equal(out[0][1].numpy(), frames[1])               # PNG: exact
    assert np.array_equal(out[0][0].numpy(), ingest.imread_gray(paths[0]))
    assert np.array_equal(out[1][0].numpy(), ingest.imread_gray(paths[2]))
