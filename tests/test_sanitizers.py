"""Host AddressSanitizer + UndefinedBehaviorSanitizer run of the CPU code this repo builds for
the host: the oracle's C restatement (every primitive the golden fixtures and GPU parity tests
rely on) and the PNG ingest library's decoder (SURVEY.md §5 "Race detection/sanitizers").  GPU
kernels cannot be sanitized on this pool; they are pinned bit for bit by the parity tests.
CPU only (gcc/g++ with -fsanitize=address,undefined)."""
import os
import shutil
import subprocess

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)


def test_oracle_and_ingest_under_asan_ubsan(tmp_path):
    gcc, gxx = shutil.which("gcc"), shutil.which("g++")
    if gcc is None or gxx is None:
        pytest.skip("gcc / g++ not available")
    san = ["-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-fno-omit-frame-pointer", "-g", "-O1"]
    objs = []
    for src in ("vo_oracle_img.c", "vo_oracle_geom.c", "vo_oracle_sift.c"):
        o = str(tmp_path / (src + ".o"))
        subprocess.run([gcc, *san, "-ffp-contract=off", "-std=gnu11", "-c", os.path.join(REPO, "oracle", src), "-o", o],
                       check=True)
        objs.append(o)
    ing = str(tmp_path / "vo_ingest.o")
    subprocess.run([gxx, *san, "-std=c++17", "-c",
                    os.path.join(REPO, "monocular_visual_odometry_va4mr_amd", "csrc", "vo_ingest.cpp"), "-o", ing],
                   check=True)
    exe = str(tmp_path / "sanitize_driver")
    subprocess.run([gxx, *san, "-std=c++17", os.path.join(HERE, "cxx", "sanitize_driver.cpp"), *objs, ing, "-o", exe,
                    "-lz", "-lpthread", "-lm"], check=True)
    from PIL import Image
    png = str(tmp_path / "frame.png")
    rng = np.random.default_rng(0)
    Image.fromarray(rng.integers(0, 256, (37, 53), dtype=np.uint8)).save(png)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", UBSAN_OPTIONS="print_stacktrace=1")
    env.pop("LD_PRELOAD", None)
    r = subprocess.run([exe, png], capture_output=True, text=True, env=env, timeout=600)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    assert r.stdout.startswith("ok"), r.stdout
