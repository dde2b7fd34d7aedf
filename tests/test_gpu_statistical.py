"""The statistical tie of the GPU render to the REFERENCE's own estimator
(SURVEY.md 8(c) fixture 8 and 8(d)'s "statistical z-test vs the reference").

The GPU draws counter-based xorshift numbers, the reference per-row mt19937
(random_state.cpp:3-17, main.cpp:222-223), so the two images agree in
distribution, not bit for bit.  tests/golden/ref_stats.npz holds per-pixel
means and variances over R = 16 independently seeded renders of the
reference's own render_subpixel row loop (main.cpp:179-197, compiled from
/root/reference by oracle/Makefile; oracle/gen_ref_paths.py) at 64x48, 4096
spp.  The GPU renders the same frame with R = 16 counter-RNG seeds, in the
product (fast) and exact arithmetic modes; per pixel-channel a two-sample
statistic z = (m_gpu - m_ref) / sqrt(v_gpu / R + v_ref / R) (~t with about
30 degrees of freedom when the estimators agree) must satisfy:
|z| > 4.5 on at most 0.5 % of pixel-channels, |mean z| < 0.08, and the
image means within 4 standard errors -- 0.17 % (box), 0.024 % (box_mirror),
0.028 % (simple) of the image mean, from the fixture's variances: a gain or
bias error of that size anywhere in the GPU path fails.
"""
import os

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

import ptgpu  # noqa: E402

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
SEED = 0x5EED0001


def two_sample_check(mg, vg, mr, vr, runs):
    """Two-sample z over pixel-channels (equal run counts on both sides, so the
    statistic is symmetric even for the skewed per-pixel distributions)."""
    # + (1e-6)^2: the fp32 image's own resolution -- channels that are
    # constant up to double rounding in the reference (variance ~1e-32: the
    # emission 0.1 or a mirror's 0.999 seen directly) differ from the fp32
    # value by ~1e-8, which is representation, not statistics
    s = np.sqrt(vg / runs + vr / runs + 1e-12)
    const = (vg == 0) & (vr < 1e-24)
    z = (mg - mr) / s
    frac = float(np.mean(np.abs(z) > 4.5))
    zm = float(z[~const].mean())
    se = float(np.sqrt(vg.sum() / runs + vr.sum() / runs) / mg.size)
    dmean = float(mg.mean() - mr.mean())
    out = {"frac_abs_z_gt_4.5": frac, "mean_z": zm, "image_mean_diff": dmean, "image_mean_se": se,
           "constant_channels": int(const.sum())}
    assert frac <= 0.005, out
    assert abs(zm) < 0.08, out
    assert abs(dmean) < 4 * se + 1e-12, out
    return out


@pytest.mark.parametrize("exact", [False, True], ids=["fast", "exact"])
@pytest.mark.parametrize("name", ["box", "box_mirror", "simple"])
def test_gpu_matches_reference_estimator(name, exact):
    if not torch.cuda.is_available():
        pytest.fail("gpu tests need a visible MI355X")
    z = np.load(os.path.join(GOLDEN, "ref_stats.npz"), allow_pickle=False)
    W, H, samps, runs = (int(z[k]) for k in ("w", "h", "samps", "runs"))
    mr, vr = z[f"{name}_mean"], z[f"{name}_var"]
    scn = ptgpu.make_scene(name, W, H)
    cam = ptgpu.camera.with_config(scn.camera_parameters)
    flags = ptgpu.FLAG_EXACT_MATH if exact else 0
    out = torch.empty(H * W * 3, dtype=torch.float32, device="cuda")
    imgs = []
    with ptgpu.Context(scn, cam) as ctx:
        for r in range(runs):
            p = ptgpu.make_params(W, H, samps, 2, SEED + 0x9E3779B97F4A7C15 * (r + 1), flags=flags)
            ctx.render_device(out, p)
            imgs.append(out.cpu().numpy().reshape(H, W, 3).astype(np.float64))
    g = np.stack(imgs)
    res = two_sample_check(g.mean(0), g.var(0, ddof=1), mr, vr, runs)
    print(name, "exact" if exact else "fast", res)
