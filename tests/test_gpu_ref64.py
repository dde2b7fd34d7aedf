"""The reference-arithmetic mode (PTG_FLAG_REFERENCE_F64, csrc/ref64.hpp)
against the oracle's Mode A/xs.

Mode A/xs restates src/main.cpp:30-197 and the pt library line by line in
double (no FMA, libm), with the counter-RNG draws; ref64.hpp is the same
restatement on the GPU, one lane per sub-pixel running its samples in order.
Division and square root are correctly rounded on both sides, the only
possible per-operation differences are the last ulp of sin/cos/pow (device
math library vs glibc).  So the images agree to rounding level: the bar here
is max |diff| <= 1e-9 on the double image (the reference's own image
precision is ~1e-16; an ulp difference amplified through a chaotic path
would show as a much larger jump), plus the segment counts exactly.
"""
import os

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

import ptgpu  # noqa: E402
import pyoracle as po  # noqa: E402

SEED = 0x5EED0001
NT = max(1, min(16, int(os.environ.get("OMP_NUM_THREADS", "8"))))


def _require_gpu():
    if not torch.cuda.is_available():
        pytest.fail("gpu tests need a visible MI355X")


def _arrays(scn):
    cam = ptgpu.camera.with_config(scn.camera_parameters)
    return (cam, np.ascontiguousarray(scn.to_array().view(po.SPHERE_DT)),
            np.ascontiguousarray(cam.to_array().view(po.CAMERA_DT)))


@pytest.mark.parametrize("name,W,H,samps", [("box", 64, 48, 16), ("box_mirror", 64, 36, 16), ("simple", 80, 60, 16),
                                            ("simple", 400, 300, 16), ("synthetic:300", 48, 27, 4)])
def test_reference_f64_matches_mode_a_xs(name, W, H, samps):
    _require_gpu()
    scn = ptgpu.make_scene(name, W, H)
    cam, sp, ca = _arrays(scn)
    img = np.zeros((H * W, 3))
    ptgpu.render(scn, cam, img, W, H, samps, flags=ptgpu.FLAG_REFERENCE_F64)
    ref, rsegs = po.render_xs_f64(sp, ca, W, H, samps, 2, SEED, nthreads=NT)
    d = np.abs(img.reshape(H, W, 3) - ref)
    exact = float((d.max(axis=2) == 0).mean())
    print(f"{name} {W}x{H}x{4 * samps}: max |diff| {d.max():.3e}, pixels bit-identical {100 * exact:.2f} %")
    assert d.max() <= 1e-9, d.max()
    assert exact > 0.99
    # segment counts through the device path (float slab)
    out = torch.zeros(H * W * 3, dtype=torch.float32, device="cuda")
    segs = torch.zeros(1, dtype=torch.int64, device="cuda")
    with ptgpu.Context(scn, cam) as ctx:
        ctx.render_device(out, ptgpu.make_params(W, H, samps, flags=ptgpu.FLAG_REFERENCE_F64), segs)
        torch.cuda.synchronize()
    assert int(segs.item()) == rsegs
    assert np.array_equal(out.cpu().numpy().reshape(H, W, 3), ref.astype(np.float32))


def test_reference_f64_c3_rows():
    """C3's full frame (box_mirror 1920x1080x1024 spp) in the reference's
    arithmetic; 8 rows against Mode A/xs."""
    _require_gpu()
    W, H, samps = 1920, 1080, 256
    scn = ptgpu.make_scene("box_mirror", W, H)
    cam, sp, ca = _arrays(scn)
    out = torch.zeros(H * W * 3, dtype=torch.float32, device="cuda")
    with ptgpu.Context(scn, cam) as ctx:
        ctx.render_device(out, ptgpu.make_params(W, H, samps, flags=ptgpu.FLAG_REFERENCE_F64))
        torch.cuda.synchronize()
    gpu = out.cpu().numpy().reshape(H, W, 3)
    ys = np.arange(67, H, 135)
    ref, _ = po.render_xs_f64(sp, ca, W, H, samps, 2, SEED, rows=(67, H, 135), nthreads=NT)
    d = np.abs(gpu[H - 1 - ys].astype(np.float64) - ref[H - 1 - ys].astype(np.float32))
    assert d.max() <= 1e-6, d.max()  # float slab: equal up to one rounding of the same double


def test_reference_f64_rejects_fp32_only_paths():
    _require_gpu()
    scn = ptgpu.box_scene(16, 8)
    cam = ptgpu.camera.with_config(scn.camera_parameters)
    p = ptgpu.make_params(16, 8, 4, flags=ptgpu.FLAG_REFERENCE_F64)
    with ptgpu.Context(scn, cam) as ctx:
        with pytest.raises(ptgpu.PtgError, match="fp32"):
            ctx.accumulate(p, 0, 2)
        with pytest.raises(ptgpu.PtgError, match="fp32"):
            ctx.trace_samples(torch.zeros((2, 5), dtype=torch.int32, device="cuda"), p)
