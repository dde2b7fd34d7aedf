"""The 4-wide BVH walk's control flow on the CPU (tools/wide_stack_depth.cpp
restates the kernel's node step: nearest hit child next, one more hit pushed
as itself, several as a (node, slot) position, a two-entry stack dropped on
overflow and the walk resumed through the continuation chain,
csrc/bvh_build.hpp wide_conts).  For every ray the nearest hit must equal an
unbounded-stack walk's, on C5's scene and on an overlap-heavy cluster where
the stack overflows often.  (The GPU parity tests check the kernel itself,
bit for bit against the oracle's linear scan.)"""
import os
import re
import shutil
import subprocess

import pytest

from conftest import ROOT
from wide_scenes import cluster_scene, dump_scene

import ptgpu


@pytest.fixture(scope="module")
def sim(tmp_path_factory):
    if shutil.which("g++") is None:
        pytest.skip("needs g++")
    exe = str(tmp_path_factory.mktemp("wsd") / "wide_stack_depth")
    subprocess.check_call(["g++", "-std=c++17", "-O2", "-I", os.path.join(ROOT, "include"),
                           os.path.join(ROOT, "tools", "wide_stack_depth.cpp"), "-o", exe])
    return exe


@pytest.mark.parametrize("name", ["synthetic:3000", "cluster"])
def test_short_stack_walk_matches_unbounded_walk(sim, tmp_path, name):
    scn = cluster_scene(1500, 64, 36) if name == "cluster" else ptgpu.make_scene(name, 64, 36)
    path = str(tmp_path / "scene.bin")
    dump_scene(scn, path)
    out = subprocess.run([sim, path, "20000"], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr
    text = out.stdout
    assert "nearest-hit mismatches vs the full walk: 0" in text, text
    over = {int(m.group(1)): float(m.group(2))
            for m in re.finditer(r"short stack (\d): node steps per ray [\d.]+, rays overflowing ([\d.]+)", text)}
    assert set(over) == {1, 2, 3, 4}
    assert over[2] > 0.05, text  # the kernel's two-entry stack overflows: the fallback is exercised
