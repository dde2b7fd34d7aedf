"""Pin the oracle (oracle/pt_oracle.c) against golden vectors produced by the
REFERENCE's own `pt` library (oracle/ref_golden.cpp built against
/root/reference/src; fixtures in tests/golden/).  All comparisons are
bit-exact: these are the reference's double-precision L0 functions.
"""
import numpy as np
import pytest

import pyoracle as po

SCENE_SIZES = {"box": ["1024x768", "1920x1080", "3840x2160"],
               "box_mirror": ["1024x768", "1920x1080", "3840x2160"],
               "simple": ["400x300"]}


def test_struct_sizes_match_reference(golden):
    sz = golden["box"]["sizeof"]
    assert sz == {"sphere": po.SPHERE_DT.itemsize, "camera": po.CAMERA_DT.itemsize,
                  "camera_config": po.CAMCFG_DT.itemsize, "vec3": 24}


def test_mt19937_generate_canonical_bitexact(golden):
    # random_state.cpp:9-17 over > 624 words (crosses a twist)
    for rec in golden["box"]["rng"]:
        g = po.MT19937(rec["seed"])
        got = [g.generate() for _ in range(len(rec["generate"]))]
        assert got == rec["generate"], rec["seed"]
        got_b = [g.generate_between(-1.0, 1.0) for _ in range(len(rec["between"]))]
        assert got_b == rec["between"]


def test_utils_bitexact(golden):
    for rec in golden["box"]["utils"]:
        assert po.lib().po_clamp(rec["x"]) == rec["clamp"]
        assert po.lib().po_color_to_int(rec["x"]) == rec["color_to_int"]


@pytest.mark.parametrize("name", ["box", "box_mirror", "simple"])
def test_scene_and_camera_bitexact(golden, name):
    for tag in SCENE_SIZES[name]:
        ref = golden[name]["scene_" + tag]
        sp, cfg = po.scene(name, ref["w"], ref["h"])
        assert len(sp) == len(ref["spheres"])
        for s, r in zip(sp, ref["spheres"]):
            assert s["radius"] == r["radius"]
            assert list(s["position"]) == r["position"]
            assert list(s["emission"]) == r["emission"]
            assert list(s["color"]) == r["color"]
            assert int(s["material"]) == r["material"]
        for k, v in ref["camera_config"].items():
            got = cfg[0][k]
            assert (list(got) if np.ndim(got) else float(got)) == v, k
        cam = po.camera_with_config(cfg)
        for k, v in ref["camera"].items():
            got = cam[0][k]
            assert (list(got) if np.ndim(got) else float(got)) == v, k


@pytest.mark.parametrize("name", ["box", "box_mirror", "simple"])
def test_sphere_intersect_and_hit_record_bitexact(golden, name):
    g = golden[name]
    tag = SCENE_SIZES[name][0]
    ref_scene = g["scene_" + tag]
    sp, _ = po.scene(name, ref_scene["w"], ref_scene["h"])
    nhit = 0
    for rec in g["intersect"]:
        s = sp[rec["i"]]
        t = po.sphere_intersect(s, rec["o"], rec["d"])
        assert t == rec["t"], rec
        if rec["t"] > 0:
            nhit += 1
            hr = po.hit_record(s, rec["o"], rec["d"], t)
            assert list(hr[0:3]) == rec["p"]
            assert list(hr[3:6]) == rec["on"]
            assert list(hr[6:9]) == rec["n"]
            assert int(hr[9]) == rec["front"]
    assert nhit > 50


@pytest.mark.parametrize("name", ["box", "box_mirror", "simple"])
def test_camera_get_ray_bitexact(golden, name):
    g = golden[name]
    ref_scene = g["scene_" + SCENE_SIZES[name][0]]
    _, cfg = po.scene(name, ref_scene["w"], ref_scene["h"])
    cam = po.camera_with_config(cfg)
    for rec in g["get_ray"]:
        rng = po.MT19937(rec["seed"])
        o, d, _ = po.get_ray(cam, rec["s"], rec["t"], rng)
        assert list(o) == rec["origin"]
        assert list(d) == rec["direction"]
        # the same number of draws was consumed (rejection loop camera.cpp:19-30)
        assert rng.generate() == rec["next"]


def test_synthetic_scene_generator_is_deterministic():
    a, ca = po.synthetic_scene(1000, 1920, 1080, 42)
    b, cb = po.synthetic_scene(1000, 1920, 1080, 42)
    assert a.tobytes() == b.tobytes() and ca.tobytes() == cb.tobytes()
    mats = np.bincount(a["material"][2:], minlength=3) / 998.0
    assert abs(mats[0] - 0.80) < 0.05 and abs(mats[1] - 0.15) < 0.04
