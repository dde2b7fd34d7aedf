"""GPU image vs the reference's arithmetic (VERDICT r1 "what's missing" 1).

test_gpu_parity.py pins the kernel to the oracle's Mode B bit for bit; Mode B
is the kernel's own fp32 op sequence.  Here the HIP image is compared with
Mode A/xs instead: the reference's double-precision arithmetic, restated line
by line from main.cpp:30-197 and the pt library (no kernel reformulation),
fed the same counter-RNG draws.  The bar is the north star's per-pixel RMSE <
1e-3 on the float image (post-clamp, pre-gamma) at every BASELINE config the
oracle finishes in seconds; each config also carries a regression guard at
about 3x the measured value (DESIGN.md "error budget").

C4 and C5 are checked at their own sample counts (4096 / 1024 spp) in
tests/test_gpu_baseline_configs.py.

Both arithmetic modes are held to the bar: the default (the GPU's own
v_sqrt/v_rsq/v_rcp/v_sin/v_cos) and PTG_FLAG_EXACT_MATH (deterministic
sequences, bit for bit Mode B -- the tests that compare with Mode B or its
segment counts use that mode).
"""
import os

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

import ptgpu  # noqa: E402
import pyoracle as po  # noqa: E402

SEED = 0x5EED0001
NORTH_STAR_RMSE = 1e-3
EXACT = ptgpu.FLAG_EXACT_MATH
NT = max(1, min(16, int(os.environ.get("OMP_NUM_THREADS", "8"))))


def _require_gpu():
    if not torch.cuda.is_available():
        pytest.fail("gpu tests need a visible MI355X")


def _arrays(scn):
    cam = ptgpu.camera.with_config(scn.camera_parameters)
    return (cam, np.ascontiguousarray(scn.to_array().view(po.SPHERE_DT)),
            np.ascontiguousarray(cam.to_array().view(po.CAMERA_DT)))


def _render(scn, cam, W, H, samps, flags=EXACT, counters=None):
    p = ptgpu.make_params(W, H, samps, 2, SEED, flags=flags)
    out = torch.full((H * W * 3,), -7.0, dtype=torch.float32, device="cuda")
    with ptgpu.Context(scn, cam) as ctx:
        ctx.render_device(out, p, counters)
        torch.cuda.synchronize()
    return out.cpu().numpy().reshape(H, W, 3)


# config, scene, W, H, samples per sub-pixel, row step, regression guard
# (measured RMSE vs Mode A/xs on these rows, exact mode: C1 5.8e-5 - 1.8e-4 (single diverging
# paths of the 30-emission light move it by ~1e-4 each), C2 3.0e-4, C3 5.0e-5)
CONFIGS = [("C1", "simple", 400, 300, 16, 1, 5e-4),
           ("C2", "box", 1024, 768, 64, 16, 9e-4),
           ("C3", "box_mirror", 1920, 1080, 256, 67, 3e-4)]
MODES = [pytest.param(EXACT, id="exact"), pytest.param(0, id="fast")]


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("cfg,name,W,H,samps,ystep,guard", CONFIGS)
def test_image_vs_reference_arithmetic(cfg, name, W, H, samps, ystep, guard, mode):
    _require_gpu()
    scn = ptgpu.make_scene(name, W, H)
    cam, sp, ca = _arrays(scn)
    gpu = _render(scn, cam, W, H, samps, flags=mode)
    y0 = ystep // 2 if ystep > 1 else 0
    ys = np.arange(y0, H, ystep)  # image-space y (main.cpp:181: y = 0 is the bottom row)
    a, _ = po.render_xs_f64(sp, ca, W, H, samps, 2, SEED, rows=(y0, H, ystep), nthreads=NT)
    g = gpu[H - 1 - ys].astype(np.float64)
    rmse = float(np.sqrt(((g - a[H - 1 - ys]) ** 2).mean()))
    assert rmse < NORTH_STAR_RMSE, (cfg, rmse)
    assert rmse < guard, (cfg, rmse)
    if cfg in ("C1", "C2") and mode == EXACT:
        # and the WHOLE frame equals the fp32 restatement (Mode B) bit for bit:
        # C1's 300 rows, C2's 768 (C3's whole frame in
        # test_c3_exact_whole_frame_bit_exact)
        b, _ = po.render_xs_f32(sp, ca, W, H, samps, 2, SEED, nthreads=NT)
        assert np.array_equal(gpu, b), (cfg, int((gpu != b).any(axis=2).sum()), "pixels differ")


_C3_FRAME = {}


@pytest.mark.parametrize("part", range(8))
def test_c3_exact_whole_frame_bit_exact(part):
    """C3 (box_mirror 1920x1080 at 1024 spp, the deep-bounce config) in the
    exact arithmetic mode: the WHOLE frame equals the fp32 restatement (Mode
    B) bit for bit.  The 1,080 rows are checked in 8
    interleaved parts (rows part, part + 8, ...: 135 rows, all their samples,
    ~30 s of CPU each on the box's 16 threads), so the suite reports progress
    between them; the GPU frame is rendered once."""
    _require_gpu()
    W, H, samps, ystep = 1920, 1080, 256, 8
    scn = ptgpu.make_scene("box_mirror", W, H)
    cam, sp, ca = _arrays(scn)
    if "gpu" not in _C3_FRAME:
        _C3_FRAME["gpu"] = _render(scn, cam, W, H, samps, flags=EXACT)
    gpu = _C3_FRAME["gpu"]
    ys = np.arange(part, H, ystep)  # image-space y
    b, _ = po.render_xs_f32(sp, ca, W, H, samps, 2, SEED, rows=(part, H, ystep), nthreads=NT)
    g, r = gpu[H - 1 - ys], b[H - 1 - ys]
    assert np.array_equal(g, r), (part, int((g != r).any(axis=2).sum()))


@pytest.mark.parametrize("name", ["box", "box_mirror", "simple", "synthetic:300"])
def test_no_out_of_range_radiance(name):
    """PTG_FLAG_COUNT_NONFINITE: no path of the shipped scenes has a NaN,
    negative or > 2^30 radiance component (the exact accumulation would clip
    it silently); the oracle counts the same."""
    _require_gpu()
    W, H, samps = 96, 64, 16
    scn = ptgpu.make_scene(name, W, H)
    cam, sp, ca = _arrays(scn)
    cnt = torch.zeros(4, dtype=torch.int64, device="cuda")
    _render(scn, cam, W, H, samps, ptgpu.FLAG_COUNT_TESTS | ptgpu.FLAG_COUNT_NONFINITE | EXACT, cnt)
    segs, _, _, bad = (int(v) for v in cnt.cpu().tolist())
    _, rsegs, rbad = po.render_xs_f32_count(sp, ca, W, H, samps, 2, SEED, nthreads=NT)
    assert segs == rsegs and bad == rbad == 0


def test_out_of_range_radiance_is_counted():
    """A light with negative emission: the counter sees every such path, the
    same number as the oracle, and the image still equals the oracle's."""
    _require_gpu()
    W, H, samps = 64, 48, 8
    scn = ptgpu.make_scene("box", W, H)
    lt = scn.spheres[5]
    scn.spheres[5] = ptgpu.sphere(lt.radius, lt.position, (-9.0, -9.0, -9.0), lt.color, lt.reflection)
    cam, sp, ca = _arrays(scn)
    cnt = torch.zeros(4, dtype=torch.int64, device="cuda")
    gpu = _render(scn, cam, W, H, samps, ptgpu.FLAG_COUNT_NONFINITE | EXACT, cnt)
    ref, _, rbad = po.render_xs_f32_count(sp, ca, W, H, samps, 2, SEED, nthreads=NT)
    assert int(cnt[3].item()) == rbad > 0
    assert np.array_equal(gpu, ref)


def test_box_mode_parallel_ray_scene():
    """camera rays with d.x == 0 exactly in a room whose
    only walls are a left/right pair (oracle/asan_check.c builds the same
    case) -- no reachable wall plane on any axis the ray moves toward.  The
    kernel masks the wall test instead of reading before the records; every
    path equals the oracle's bit for bit."""
    _require_gpu()
    R, off = 1e6, 0.4
    spheres = [ptgpu.sphere(R, (-R - off, 0.0, -1.0), (0, 0, 0), (0.9, 0.1, 0.2), ptgpu.reflection_type.diffuse),
               ptgpu.sphere(R, (R + off, 0.0, -1.0), (0, 0, 0), (0.3, 0.1, 0.9), ptgpu.reflection_type.diffuse),
               ptgpu.sphere(0.2, (0.0, -0.2, -1.0), (0, 0, 0), (1, 1, 1), ptgpu.reflection_type.specular)]
    W, H, nsub = 1 << 19, 1, 8
    cfg = ptgpu.camera_config()
    cfg.position = (0.0, 0.0, 2.0)
    cfg.direction = (0.0, 0.0, -1.0)
    cfg.up = (0.0, 1.0, 0.0)
    cfg.aspect_ratio = W / H
    cfg.vertical_fov_radians = 0.5
    cfg.aperture = 0.0
    cfg.focus_distance = 3.0
    scn = ptgpu.scene(spheres, cfg)
    cam, sp, ca = _arrays(scn)
    assert po.scan_layout(sp, ca)[0][:2] == [3, 3]
    coords = np.array([[W // 2, 0, 0, sy, k] for sy in range(nsub) for k in range(256)], dtype=np.int32)
    p = ptgpu.make_params(W, H, 1, nsub, SEED, flags=EXACT)
    with ptgpu.Context(scn, cam) as ctx:
        out, segs = ctx.trace_samples(torch.from_numpy(coords).cuda(), p)
    out = out.cpu().numpy()
    segs = segs.cpu().numpy()
    for i, (x, y, sx, sy, k) in enumerate(coords):
        ref, rs = po.sample_f32(sp, ca, W, H, nsub, SEED, int(x), int(y), int(sx), int(sy), int(k))
        assert segs[i] == rs and out[i].tobytes() == ref.tobytes(), (i, out[i], ref)


def test_one_shot_render_after_progressive_passes():
    """accumulate + keep_acc resolve leave progressive
    sums in the context's accumulator; a later one-shot render on the same
    context must not add them in (it clears them first).  Checked on a frame
    with a split tail and on a chunked one (the default arithmetic mode)."""
    _require_gpu()
    for W, H, samps, chunk in ((1920, 1080, 8, 0), (40, 24, 16, 3)):
        scn = ptgpu.box_scene(W, H)
        cam = ptgpu.camera.with_config(scn.camera_parameters)
        p = ptgpu.make_params(W, H, samps, 2, SEED, chunk_samples=chunk)
        fresh = _render(scn, cam, W, H, samps, flags=0) if chunk == 0 else None
        out = torch.empty(H * W * 3, dtype=torch.float32, device="cuda")
        with ptgpu.Context(scn, cam) as ctx:
            ctx.reset_accumulation(p)
            ctx.accumulate(p, 0, 5)
            ctx.resolve(out, p, 5)
            ctx.render_device(out, p)
            torch.cuda.synchronize()
            img = out.cpu().numpy().reshape(H, W, 3)
            ctx.render_device(out, p)  # and again: the buffer stays clean
            torch.cuda.synchronize()
            again = out.cpu().numpy().reshape(H, W, 3)
        if fresh is None:
            fresh = _render_chunked(scn, cam, W, H, samps, chunk)
        assert np.array_equal(img, fresh) and np.array_equal(again, fresh)


def _render_chunked(scn, cam, W, H, samps, chunk):
    p = ptgpu.make_params(W, H, samps, 2, SEED, chunk_samples=chunk)
    out = torch.empty(H * W * 3, dtype=torch.float32, device="cuda")
    with ptgpu.Context(scn, cam) as ctx:
        ctx.render_device(out, p)
        torch.cuda.synchronize()
    return out.cpu().numpy().reshape(H, W, 3)


def test_too_many_work_units_fail_loudly():
    """the grid is computed in 64 bits; a chunk size that
    would need more than 2^31 - 1 workgroups is rejected, nothing launches."""
    _require_gpu()
    W, H = 1920, 1080
    scn = ptgpu.box_scene(W, H)
    cam = ptgpu.camera.with_config(scn.camera_parameters)
    out = torch.full((H * W * 3,), -7.0, dtype=torch.float32, device="cuda")
    with ptgpu.Context(scn, cam) as ctx:
        with pytest.raises(ptgpu.PtgError, match="too many work units"):
            ctx.render_device(out, ptgpu.make_params(W, H, 1 << 28, 2, SEED, chunk_samples=1))
        torch.cuda.synchronize()
    assert (out == -7.0).all()


def test_context_checks_tensors():
    """trace_samples needs int32 [n, 5] coordinates and
    every tensor must sit on the context's device."""
    _require_gpu()
    scn = ptgpu.box_scene(8, 8)
    cam = ptgpu.camera.with_config(scn.camera_parameters)
    p = ptgpu.make_params(8, 8, 1)
    with ptgpu.Context(scn, cam, device=0) as ctx:
        assert ctx.device == 0
        with pytest.raises(ValueError):
            ctx.trace_samples(torch.zeros((4, 5), dtype=torch.int64, device="cuda"), p)
        with pytest.raises(ValueError):
            ctx.trace_samples(torch.zeros((4, 4), dtype=torch.int32, device="cuda"), p)
        with pytest.raises(ValueError):
            ctx.render_device(torch.zeros(8 * 8 * 3, dtype=torch.float64, device="cuda"), p)


def test_sunk_spheres_image_bitexact():
    """Glass spheres sunk into the walls (tests/test_wall_rules.py): the GPU
    keeps wall pairs and box mode and equals the oracle bit for bit."""
    _require_gpu()
    from test_wall_rules import sunk_scene
    W, H, samps = 64, 48, 16
    scn = sunk_scene(W, H)
    cam, sp, ca = _arrays(scn)
    gpu = _render(scn, cam, W, H, samps)
    ref, _ = po.render_xs_f32(sp, ca, W, H, samps, 2, SEED, nthreads=NT)
    assert np.array_equal(gpu, ref)


@pytest.mark.gpu
def test_fresh_contexts_on_side_streams():
    """A fresh context's first frame on a non-blocking stream (torch side
    streams are created non-blocking): the accumulator's first zeroing is
    queued on that stream (ensure_acc), not on the null stream, which such a
    stream does not wait for.  Frames with an HBM-accumulated split tail and
    with sample chunks, several fresh contexts each, equal the frame rendered
    on the current stream bit for bit."""
    _require_gpu()
    for W, H, samps, chunk in ((1920, 1080, 4, 0), (48, 30, 16, 3)):
        scn = ptgpu.box_mirror_scene(W, H)
        cam = ptgpu.camera.with_config(scn.camera_parameters)
        p = ptgpu.make_params(W, H, samps, 2, SEED, chunk_samples=chunk)
        ref = _render_chunked(scn, cam, W, H, samps, chunk)
        for _ in range(4):
            side = torch.cuda.Stream()
            out = torch.full((H * W * 3,), -7.0, dtype=torch.float32, device="cuda")
            torch.cuda.synchronize()
            with ptgpu.Context(scn, cam) as ctx:
                ctx.render_device(out, p, stream=side)
                side.synchronize()
            assert np.array_equal(out.cpu().numpy().reshape(H, W, 3), ref)
