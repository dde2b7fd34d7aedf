"""Runtime scene files (the reference hard-codes its scene,
main.cpp:25,199-208): the Python reader/writer (ptgpu.scene) and the C++ CLI's
(host/pt/scene_file.hpp) agree with each other and with the built-in scenes
bit for bit; malformed files fail loudly.  No GPU work: the CLI runs with
--no-render."""
import json
import os
import subprocess

import numpy as np
import pytest

import ptgpu
from conftest import ROOT

CLI = os.path.join(ROOT, "cpu-path-tracing_amd", "pt_render_gpu")


def _cli(*args):
    return subprocess.run([CLI, *args], capture_output=True, text=True, timeout=60)


def _dump(scene_arg, w, h, tmp_path):
    out = tmp_path / "dump.json"
    r = _cli("--scene", scene_arg, "--width", str(w), "--height", str(h), "--dump-json", str(out), "--no-render")
    assert r.returncode == 0, r.stderr
    return json.loads(out.read_text())


def _py_dump(scn):
    cam = ptgpu.camera.with_config(scn.camera_parameters)
    return scn.to_array(), cam.to_array()


def _check_same(d, scn):
    sp, ca = _py_dump(scn)
    assert len(d["spheres"]) == len(sp)
    for rec, s in zip(d["spheres"], sp):
        assert rec["radius"] == s["radius"] and rec["material"] == s["material"]
        for k in ("position", "emission", "color"):
            assert rec[k] == list(s[k]), k
    for k in ("position", "lower_left_corner", "cam_x_axis", "cam_y_axis", "u", "v", "w"):
        assert d["camera"][k] == list(ca[0][k]), k
    assert d["camera"]["lens_radius"] == ca[0]["lens_radius"]


@pytest.mark.parametrize("name", ["box", "box_mirror", "simple", "synthetic:300"])
def test_python_round_trip_is_exact(name, tmp_path):
    scn = ptgpu.make_scene(name, 200, 150)
    path = tmp_path / "s.scene"
    ptgpu.save_scene_file(scn, str(path))
    back = ptgpu.load_scene_file(str(path), 200, 150)
    assert np.array_equal(back.to_array(), scn.to_array())
    assert back.camera_parameters == scn.camera_parameters
    assert ptgpu.make_scene(str(path), 200, 150).camera_parameters == scn.camera_parameters


@pytest.mark.parametrize("name", ["box", "box_mirror", "simple", "synthetic:40"])
def test_cli_and_python_agree(name, tmp_path):
    """The C++ CLI's built-in scenes, its scene-file writer and reader, and the
    Python side all give the same spheres and camera::with_config result."""
    w, h = 320, 180
    scn = ptgpu.make_scene(name, w, h)
    _check_same(_dump(name, w, h, tmp_path), scn)
    saved = tmp_path / "cli.scene"
    r = _cli("--scene", name, "--width", str(w), "--height", str(h), "--save-scene", str(saved), "--no-render")
    assert r.returncode == 0, r.stderr
    assert saved.read_text() == ptgpu.scene_text(scn)  # identical writers
    _check_same(_dump(str(saved), w, h, tmp_path), scn)


HAND_WRITTEN = """
# a hand-written scene: comments, blank lines, exponents, auto focus
camera 0 1 4   0 0.5 -1   0 1 0   0.7 0.1 auto   # pos look-at up vfov aperture focus

sphere 1e3   0 -1000 0    0 0 0        0.5 0.5 0.5   diffuse
sphere 0.5   -1 0.5 -1    0 0 0        1 1 1         dielectric
sphere 0.5   1 0.5 -1     0 0 0        0.9 0.9 0.9   specular
sphere 0.25  0 2.5 -1     12 12 12     0 0 0         diffuse
"""


def test_hand_written_file(tmp_path):
    path = tmp_path / "hand.scene"
    path.write_text(HAND_WRITTEN)
    scn = ptgpu.load_scene_file(str(path), 640, 360)
    assert len(scn.spheres) == 4
    c = scn.camera_parameters
    assert c.aspect_ratio == 640 / 360 and c.focus_distance == ptgpu.length((0.0, 0.5, 5.0))
    assert [int(s.reflection) for s in scn.spheres] == [0, 2, 1, 0]
    _check_same(_dump(str(path), 640, 360, tmp_path), scn)


BAD = {
    "unknown": ("camera 0 0 2 0 0 0 0 1 0 0.5 0 auto\ncube 1 2 3\n", "line 2: unknown item"),
    "count": ("camera 0 0 2 0 0 0 0 1 0 0.5 0 auto\nsphere 1 0 0 0 0 0 0 1 1 diffuse\n", "line 2: sphere needs"),
    "number": ("camera 0 0 2 0 0 0 0 1 0 0.5 0 auto\nsphere 1 0 0 x 0 0 0 1 1 1 diffuse\n", "line 2: not a number"),
    "material": ("camera 0 0 2 0 0 0 0 1 0 0.5 0 auto\nsphere 1 0 0 0 0 0 0 1 1 1 metal\n", "line 2: material"),
    "radius": ("camera 0 0 2 0 0 0 0 1 0 0.5 0 auto\nsphere -1 0 0 0 0 0 0 1 1 1 diffuse\n", "line 2: radius"),
    "focus": ("camera 0 0 2 0 0 0 0 1 0 0.5 0 near\n", "line 1: focus"),
    "no_camera": ("sphere 1 0 0 0 0 0 0 1 1 1 diffuse\n", "no camera"),
    "two_cameras": ("camera 0 0 2 0 0 0 0 1 0 0.5 0 auto\ncamera 0 0 2 0 0 0 0 1 0 0.5 0 auto\n", "line 2: second camera"),
}


@pytest.mark.parametrize("case", sorted(BAD))
def test_malformed_files_fail_loudly(case, tmp_path):
    text, msg = BAD[case]
    path = tmp_path / f"{case}.scene"
    path.write_text(text)
    with pytest.raises(ptgpu.SceneFileError, match=msg):
        ptgpu.load_scene_file(str(path), 64, 48)
    r = _cli("--scene", str(path), "--no-render")
    assert r.returncode == 2 and msg in r.stderr, r.stderr


def test_cli_rejects_bad_options():
    assert _cli("--bogus").returncode == 2
    assert _cli("--width", "0", "--no-render").returncode == 2
    assert _cli("--scene", "/nonexistent.scene", "--no-render").returncode == 2
