"""Box mode's degenerate case under AddressSanitizer.

oracle/asan_check.c renders, through the oracle's Mode B, camera rays with
d.x == 0 exactly in a scene whose only walls are a left/right pair: no axis
the ray moves toward has a reachable wall plane.  Round 1 then selected a
missing wall and read the record before the scene array (reproduced with this
driver: heap-buffer read in test_B via box_walls_B); the kernel had the same
selection (ptg_render.hip scene_scan).  Both now mask the test; this build
runs the driver with ASan + UBSan and requires a clean exit.  The GPU side of
the same rays: test_gpu_reference.py::test_box_mode_parallel_ray_scene.
"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_box_mode_parallel_rays_asan(tmp_path):
    if shutil.which("gcc") is None:
        pytest.skip("gcc not available")
    exe = tmp_path / "asan_check"
    odir = os.path.join(ROOT, "oracle")
    cmd = ["gcc", "-std=c11", "-O1", "-g", "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
           "-fno-omit-frame-pointer", "-ffp-contract=off", "-fopenmp", "-I", odir,
           os.path.join(odir, "asan_check.c"), os.path.join(odir, "pt_oracle.c"), "-lm", "-o", str(exe)]
    subprocess.check_call(cmd)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=0", OMP_NUM_THREADS="1")
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.startswith("ok "), r.stdout
