"""CPU tests of the host side: the C ABI library loads and exports every
declared symbol, the host mirrors of the reference's scenes/camera are
bit-exact against the compiled reference's dumps, shard geometry, and the
error behaviour of the ABI (no GPU compute is launched here)."""
import ctypes as C
import os
import re
import subprocess

import numpy as np
import pytest

import ptgpu
import pyoracle as po
from conftest import ROOT

SIZES = {"box": ["1024x768", "1920x1080", "3840x2160"], "box_mirror": ["1024x768", "1920x1080", "3840x2160"],
         "simple": ["400x300"]}


def _header_symbols():
    with open(os.path.join(ROOT, "include", "ptgpu.h")) as f:
        text = f.read()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\s*\*?\s*(ptg_\w+)\s*\(", text, re.M)))


def test_library_exports_every_declared_symbol():
    syms = _header_symbols()
    assert len(syms) == len(ptgpu.EXPORTS) and set(syms) == set(ptgpu.EXPORTS)
    lib = C.CDLL(ptgpu.LIB_PATH)
    for s in syms:
        assert hasattr(lib, s), s
    out = subprocess.run(["nm", "-D", "--defined-only", ptgpu.LIB_PATH], capture_output=True, text=True).stdout
    for s in syms:
        assert re.search(rf"\bT {s}\b", out), s
    assert ptgpu.lib().ptg_abi_version() == ptgpu.ABI_VERSION


def test_library_is_gfx950_code():
    with open(ptgpu.LIB_PATH, "rb") as f:
        blob = f.read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob


@pytest.mark.parametrize("name", ["box", "box_mirror", "simple"])
def test_host_scenes_bitexact_vs_reference(golden, name):
    for tag in SIZES[name]:
        ref = golden[name]["scene_" + tag]
        scn = ptgpu.make_scene(name, ref["w"], ref["h"])
        arr = scn.to_array()
        assert len(arr) == len(ref["spheres"])
        for s, r in zip(arr, ref["spheres"]):
            assert float(s["radius"]) == r["radius"]
            assert list(s["position"]) == r["position"]
            assert list(s["emission"]) == r["emission"]
            assert list(s["color"]) == r["color"]
            assert int(s["material"]) == r["material"]
        c = scn.camera_parameters
        for k, v in ref["camera_config"].items():
            got = getattr(c, k)
            assert (list(got) if isinstance(got, tuple) else got) == v, k
        cam = ptgpu.camera.with_config(c)
        for k, v in ref["camera"].items():
            got = getattr(cam, k)
            assert (list(got) if isinstance(got, tuple) else got) == v, k


def test_synthetic_scene_matches_oracle_generator():
    scn = ptgpu.synthetic_scene(500, 1920, 1080, 42)
    ref, cfg = po.synthetic_scene(500, 1920, 1080, 42)
    assert scn.to_array().tobytes() == ref.tobytes()
    c = scn.camera_parameters
    assert list(c.position) == list(cfg[0]["position"]) and c.focus_distance == cfg[0]["focus_distance"]


@pytest.mark.parametrize("H,br,count", [(1080, 8, 1), (1080, 8, 3), (1080, 8, 8), (768, 16, 4), (23, 8, 2),
                                        (7, 4, 5)])
def test_shard_rows_cover_image_exactly_once(H, br, count):
    seen = np.concatenate([ptgpu.slab_to_image_rows(H, br, k, count) for k in range(count)])
    seen = seen[seen >= 0]
    assert sorted(seen.tolist()) == list(range(H))
    W = 5
    rows = ptgpu.shard_rows(H, br, count)
    full = np.random.default_rng(0).random((H, W, 3)).astype(np.float32)
    gathered = np.zeros((count, rows, W, 3), np.float32)
    for k in range(count):
        m = ptgpu.slab_to_image_rows(H, br, k, count)
        gathered[k][m >= 0] = full[m[m >= 0]]
    assert np.array_equal(ptgpu.unshard_host(gathered, W, H, br, count), full)


def test_abi_rejects_bad_arguments_without_gpu_work():
    L = ptgpu.lib()
    out = C.c_int32()
    assert L.ptg_shard_rows(0, 8, 1, C.byref(out)) == -1
    assert L.ptg_shard_rows(1080, 8, 8, C.byref(out)) == 0 and out.value == 136
    scn = ptgpu.box_scene(8, 8)
    cam = ptgpu.camera.with_config(scn.camera_parameters)
    img = np.zeros((64, 3))
    with pytest.raises(ptgpu.PtgError, match="num_subpixels"):
        ptgpu.render(scn, cam, img, 8, 8, 4, num_subpixels=0)
    with pytest.raises(ptgpu.PtgError, match="samples"):
        ptgpu.render(scn, cam, img, 8, 8, -3)
    with pytest.raises(ValueError):
        ptgpu.render(scn, cam, np.zeros((10, 3)), 8, 8, 4)
    bad = scn.to_array()
    bad[0]["material"] = 7
    with pytest.raises(ptgpu.PtgError, match="invalid"):
        ptgpu.Context(bad, cam)


def test_multi_abi_rejects_bad_arguments_without_gpu_work():
    """ptg_multi_* / ptg_render_multi argument checks: NULL
    arguments, a frame it would have to shard twice and the
    reference-arithmetic flag are refused before any device work (here: no
    GPU at all -- create reports PTG_ERR_NO_DEVICE and leaves *out NULL)."""
    L = ptgpu.lib()
    scn = ptgpu.box_scene(8, 8)
    cam = ptgpu.camera.with_config(scn.camera_parameters)
    sp, ca = scn.to_array(), cam.to_array()
    img = np.zeros((64, 3))
    devs = (C.c_int * 2)(0, 1)
    args = (sp.ctypes.data_as(C.c_void_p), len(sp), ca.ctypes.data_as(C.c_void_p))
    p = ptgpu.make_params(8, 8, 4, flags=ptgpu.FLAG_REFERENCE_F64)
    assert L.ptg_render_multi(*args, C.byref(p), devs, 2, img.ctypes.data_as(C.c_void_p)) == -4  # UNSUPPORTED
    assert b"fp32 kernel only" in L.ptg_last_error()
    p = ptgpu.make_params(8, 8, 4, shard_rank=1, shard_count=2)
    assert L.ptg_render_multi(*args, C.byref(p), devs, 2, img.ctypes.data_as(C.c_void_p)) == -1
    p = ptgpu.make_params(8, 8, 4)
    assert L.ptg_render_multi(*args, C.byref(p), devs, 0, img.ctypes.data_as(C.c_void_p)) == -1
    assert L.ptg_multi_render(None, C.byref(p), img.ctypes.data_as(C.c_void_p)) == -1
    assert L.ptg_multi_resolve(None, C.byref(p), 0, None) == -1
    assert L.ptg_multi_destroy(None) == 0
    h = C.c_void_p(1)
    rc = L.ptg_multi_create(*args, devs, 2, C.byref(h))
    n = C.c_int(0)
    L.ptg_device_count(C.byref(n))
    if n.value == 0:  # the CPU container: no device, nothing created
        assert rc == -3 and not h.value


def _tilted_box():
    scn = ptgpu.make_scene("box", 64, 48)
    R = 1e6
    k = R / 2 ** 0.5
    tilted = ptgpu.sphere(R, (k + 0.3, 0.0, -k - 0.3), (0.0, 0.0, 0.0), (0.2, 0.6, 0.6),
                          ptgpu.reflection_type.specular)
    scn.spheres = scn.spheres[5:] + [tilted] + scn.spheres[:5]
    return scn


@pytest.mark.parametrize("name", ["box", "box_mirror", "simple", "synthetic:40", "synthetic:300", "tilted"])
def test_scene_layout_matches_oracle(name):
    """The kernel host's anchor choice and scan order (ptg_scene_layout, no GPU)
    equal the oracle's Mode B preparation: the box walls take the axis
    anchors, a 45-degree huge sphere keeps the camera-facing anchor."""
    scn = _tilted_box() if name == "tilted" else ptgpu.make_scene(name, 64, 48)
    cam = ptgpu.camera.with_config(scn.camera_parameters)
    axis, order = ptgpu.scene_layout(scn, cam)
    sp = scn.to_array().view(po.SPHERE_DT)
    ca = cam.to_array().view(po.CAMERA_DT)
    assert (axis, order) == po.scan_layout(sp, ca)
    assert sorted(order) == list(range(len(scn.spheres)))
    # axis-anchored walls report their axis, wall pairs 3 + axis (+ wall first
    # in the scan: right before left, ceiling before floor); the back wall
    # has no partner
    if name in ("box", "box_mirror"):
        assert axis == [3, 3, 2, 4, 4, -1, -1, -1] and order == [1, 0, 3, 4, 2, 5, 6, 7]
    if name == "tilted":
        assert axis == [-1, -1, -1, -1, 3, 3, 2, 4, 4] and order == [5, 4, 7, 8, 6, 3, 0, 1, 2]
    if name == "simple":  # the R = 100 ground is anchored on y (is_huge: R > 16 (camera distance + 1)); index order
        assert axis == [1, -1, -1, -1, -1] and order == list(range(5))


def test_params_struct_matches_header():
    assert C.sizeof(ptgpu.Params) == 48
    p = ptgpu.make_params(1920, 1080, 256)
    assert (p.width, p.height, p.samples, p.num_subpixels, p.band_rows, p.shard_count) == (1920, 1080, 256, 2, 1, 1)
