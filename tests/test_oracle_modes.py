"""The three oracle modes estimate the same image.

Mode A/mt (reference arithmetic + mt19937 row seeding), Mode A/xs (same
arithmetic, counter xorshift) and Mode B (the GPU's fp32 op sequence) draw
different random numbers (mt vs xs) or round differently (A vs B), so they
agree statistically, not bitwise: per-pixel differences are bounded by the
Monte-Carlo error, image means agree tightly, and A/xs vs B share the
random streams so most pixels agree closely.
"""
import numpy as np
import pytest

import pyoracle as po


def _scene(name, W, H):
    sp, cfg = po.scene(name, W, H)
    return sp, po.camera_with_config(cfg)


@pytest.mark.parametrize("name", ["box", "box_mirror", "simple"])
def test_modes_agree_statistically(name):
    W, H, samps = 48, 36, 64
    sp, cam = _scene(name, W, H)
    a_mt = po.render_mt(sp, cam, W, H, samps, rd_value=12345)
    a_xs, segs_a = po.render_xs_f64(sp, cam, W, H, samps)
    b_xs, segs_b = po.render_xs_f32(sp, cam, W, H, samps)
    # image means: independent estimates (mt vs xs) within a few standard errors
    for img in (a_xs, b_xs):
        assert abs(img.mean() - a_mt.mean()) < 0.02 * max(a_mt.mean(), 0.05) + 0.004
    # same random streams: A/xs and B follow identical paths except where fp32
    # rounding flips a decision -> the north star's per-pixel RMSE < 1e-3
    # (measured at 256 spp: box 4.8e-5, box_mirror 1.8e-4, simple 3e-8), and
    # segment counts within 1 %
    rmse = float(np.sqrt(((a_xs - b_xs.astype(np.float64)) ** 2).mean()))
    assert rmse < 1e-3, rmse
    assert abs(segs_a - segs_b) / segs_a < 0.01


def test_segments_per_path_matches_survey():
    # SURVEY.md §3.5 (gprof call counts): 12.34 box, 12.40 box_mirror, 2.08 simple
    for name, expect in (("box", 12.34), ("box_mirror", 12.40), ("simple", 2.08)):
        W, H, samps = 64, 48, 16
        sp, cam = _scene(name, W, H)
        _, segs = po.render_xs_f64(sp, cam, W, H, samps)
        sbar = segs / (W * H * 4 * samps)
        assert abs(sbar - expect) / expect < 0.03, (name, sbar)


def test_radiance_mt_consumes_reference_draw_order():
    """radiance() with an mt19937 stream: a path that ends by RR consumed
    exactly one RR draw per bounce past depth 4 plus the material draws; the
    restated loop is deterministic given the seed."""
    sp, cam = _scene("box", 64, 48)
    outs = []
    for _ in range(2):
        g = po.MT19937(99)
        o, d, _ = po.get_ray(cam, 0.5, 0.5, g)
        c, segs = po.radiance_mt(sp, o, d, g)
        outs.append((tuple(c), segs, g.generate()))
    assert outs[0] == outs[1]
    assert outs[0][1] >= 6  # RR never fires before depth 5 (main.cpp:130)


def test_mode_b_sincos_table_accuracy():
    """Mode B's cos/sin(2 pi u) (256-entry table + rotation, main.cpp:55's
    libm calls restated) over EVERY 24-bit u: within 3e-7 of the double
    values, and cos^2 + sin^2 = 1 within 1e-6 (the diffuse direction stays a
    unit vector, main.cpp:55)."""
    m = np.arange(1 << 24, dtype=np.uint32)
    cs = po.sincos2pi(m).astype(np.float64)
    ang = 2.0 * np.pi * m.astype(np.float64) * 2.0 ** -24
    assert np.abs(cs[:, 0] - np.cos(ang)).max() < 3e-7
    assert np.abs(cs[:, 1] - np.sin(ang)).max() < 3e-7
    assert np.abs((cs ** 2).sum(axis=1) - 1.0).max() < 1e-6


def test_mode_b_division_and_sqrt_accuracy():
    """Mode B's deterministic division (Newton reciprocal + residual
    correction) and square root (Goldschmidt + a Newton residual step) over
    10^6 operands spanning 1e-8 .. 1e8: division within 2 ulp (measured 0.5),
    sqrt within 1.2e-7 relative (about 1 ulp; measured 0.63 ulp); sqrt of zero
    and negative values is 0."""
    rng = np.random.default_rng(11)
    n = 1_000_000
    a = (10.0 ** rng.uniform(-8, 8, n) * rng.choice([-1.0, 1.0], n)).astype(np.float32)
    b = (10.0 ** rng.uniform(-8, 8, n)).astype(np.float32)
    q, r = po.mode_b_math(a, b)
    exact = a.astype(np.float64) / b.astype(np.float64)
    ulp = np.spacing(np.abs(exact).astype(np.float32)).astype(np.float64)
    assert (np.abs(q - exact) <= 2 * ulp).all()
    pos = a > 0
    rel = np.abs(r[pos] - np.sqrt(a[pos].astype(np.float64))) / np.sqrt(a[pos].astype(np.float64))
    assert rel.max() < 1.2e-7
    assert (r[~pos] == 0).all()
    z, rz = po.mode_b_math(np.array([0.0, -0.0, 4.0], np.float32), np.ones(3, np.float32))
    assert rz[0] == 0 and rz[1] == 0 and rz[2] == 2.0


@pytest.mark.parametrize("name,W,H,samps,rows,cols", [("box", 64, 48, 4, (3, 40, 7), (5, 50)),
                                                      ("synthetic:300", 64, 36, 2, (0, 36, 5), (0, 64))])
def test_rect_renders_equal_row_renders(name, W, H, samps, rows, cols):
    """po_render_xs_*_rect (parallel over pixels, for single rows at the
    BASELINE sample counts) gives the row renders' bits on its rectangle and
    leaves the rest untouched, in both arithmetic modes."""
    import ptgpu
    scn = ptgpu.make_scene(name, W, H)
    cam = ptgpu.camera.with_config(scn.camera_parameters)
    sp = np.ascontiguousarray(scn.to_array().view(po.SPHERE_DT))
    ca = np.ascontiguousarray(cam.to_array().view(po.CAMERA_DT))
    ys = H - 1 - np.arange(*rows)
    for f64 in (False, True):
        r, _ = po.render_xs_rect(sp, ca, W, H, samps, 2, 0x5EED0001, cols=cols, rows=rows, f64=f64)
        full, _ = (po.render_xs_f64 if f64 else po.render_xs_f32)(sp, ca, W, H, samps, 2, 0x5EED0001, rows=rows)
        assert np.array_equal(r[ys][:, cols[0]:cols[1]], full[ys][:, cols[0]:cols[1]])
        mask = np.ones((H, W), bool)
        mask[np.ix_(ys, np.arange(*cols))] = False
        assert (r[mask] == 0).all() and r[~mask].sum() > 0


def test_mode_b_output_is_pinned():
    """The checker itself is pinned: Mode B frames -- the fp32
    restatement the GPU's exact mode must equal bit for bit -- against the
    values stored by oracle/gen_mode_b_pin.py, so a change of compiler or
    flags in oracle/Makefile (-O3, -mfma, -ffp-contract=off) cannot move the
    oracle without this test failing."""
    import os
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
    import gen_mode_b_pin as g
    z = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "mode_b_pin.npz"),
                allow_pickle=False)
    for name, W, H, samps in g.CASES:
        img, segs = g.frame(name, W, H, samps)
        key = name.replace(":", "_")
        assert np.array_equal(img, z[key]), name
        assert segs == int(z[key + "_segments"]), name
