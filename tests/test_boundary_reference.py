"""The C-ABI boundary against the reference's real headers.

tests/ref_boundary.cpp includes /root/reference/src's sphere/camera/scene/vec
headers and include/ptgpu.h, static_asserts every field offset of pt::sphere
and pt::camera against ptg_sphere / ptg_camera, and compiles INTEGRATION.md
section 2's casts, linked against libptgpu.so and the reference's own pt
library (oracle/_ref, built from the reference's sources).  Without a GPU
(this container) ptg_render must return PTG_ERR_NO_DEVICE cleanly and leave
the image untouched.  Needs /root/reference: skipped where it is absent (the
GPU box).
"""
import os
import subprocess

import pytest

from conftest import ROOT

REF = "/root/reference/src"


def test_reference_headers_match_the_abi(tmp_path):
    if not os.path.isdir(REF):
        pytest.skip("/root/reference not present")
    lib_ref = os.path.join(ROOT, "oracle", "_ref", "libpt_ref.a")
    if not os.path.exists(lib_ref):
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "_ref/libpt_ref.a"])
    pkg = os.path.join(ROOT, "cpu-path-tracing_amd")
    exe = tmp_path / "ref_boundary"
    subprocess.check_call(["g++", "-std=c++17", "-O1", "-Wall", "-I", REF, "-I", os.path.join(ROOT, "include"),
                           os.path.join(ROOT, "tests", "ref_boundary.cpp"), lib_ref, "-L", pkg, "-lptgpu",
                           f"-Wl,-rpath,{pkg}", "-o", str(exe)])
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "layout 0 axis 3 3 2 4 4" in r.stdout, r.stdout
