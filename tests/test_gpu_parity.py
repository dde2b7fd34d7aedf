"""GPU parity: the HIP megakernel (through the C ABI) against the oracle.

Tolerance: in its exact arithmetic mode (PTG_FLAG_EXACT_MATH) the kernel and
the oracle's Mode B execute the same fp32 op sequence, so the bar is
BIT-EXACT equality (max |diff| == 0) of images, per-path radiance and segment
counts.  The default (fast-transcendental) mode is held to the north star's
RMSE against the reference arithmetic in test_gpu_reference.py and
test_gpu_baseline_configs.py, and to the same GPU-vs-GPU invariances
(shards, work units, split tails, progressive passes) bit for bit in
test_gpu_fast_math.py.  The north-star tolerance (per-pixel
RMSE < 1e-3 on the float image, post-clamp, pre-gamma) is asserted as well
so that a future non-bit-exact kernel change fails loudly on the stated bar.
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

import ptgpu  # noqa: E402
import pyoracle as po  # noqa: E402

RMSE_TOL = 1e-3
SEED = 0x5EED0001
EXACT = ptgpu.FLAG_EXACT_MATH  # every image here is compared with Mode B bit for bit


def _require_gpu():
    if not torch.cuda.is_available():
        pytest.fail("gpu tests need a visible MI355X")
    n = __import__("ctypes").c_int(0)
    ptgpu.lib().ptg_device_count(__import__("ctypes").byref(n))
    assert n.value >= 1


def _oracle_scene(scn, cam):
    sp = scn.to_array().view(po.SPHERE_DT)
    return np.ascontiguousarray(sp), np.ascontiguousarray(cam.to_array().view(po.CAMERA_DT))


def _gpu_image(scn, cam, W, H, samps, nsub=2, seed=SEED, band_rows=8, rank=0, count=1, count_segments=False,
               chunk=0):
    p = ptgpu.make_params(W, H, samps, nsub, seed, band_rows, rank, count, chunk,
                          flags=(ptgpu.FLAG_COUNT_TESTS if count_segments else 0) | EXACT)
    rows = ptgpu.shard_rows(H, band_rows, count)
    out = torch.full((rows * W * 3,), -7.0, dtype=torch.float32, device="cuda")
    segs = torch.zeros(3, dtype=torch.int64, device="cuda") if count_segments else None
    with ptgpu.Context(scn, cam) as ctx:
        ctx.render_device(out, p, segs)
        torch.cuda.synchronize()
    img = out.cpu().numpy().reshape(rows, W, 3)
    if count == 1:
        img = img[:H]
    if segs is not None:
        _gpu_image.tests = segs.cpu().tolist()
    return img, (int(segs[0].item()) if segs is not None else None)


def _check_equal(gpu, ref):
    diff = np.abs(gpu.astype(np.float64) - ref.astype(np.float64))
    rmse = float(np.sqrt((diff ** 2).mean()))
    assert rmse < RMSE_TOL, rmse
    assert float(diff.max()) == 0.0, (float(diff.max()), int((diff > 0).sum()))


# > 64 spheres: BVH traversal on the GPU, linear scan with the same nearest-hit rule in the oracle
CASES = [("box", 64, 48, 16), ("box_mirror", 64, 36, 16), ("simple", 80, 60, 16), ("synthetic:300", 64, 36, 8),
         ("synthetic:10000", 48, 27, 4)]


@pytest.mark.parametrize("name,W,H,samps", CASES)
def test_image_bitexact_vs_oracle(name, W, H, samps):
    _require_gpu()
    scn = ptgpu.make_scene(name, W, H)
    cam = ptgpu.camera.with_config(scn.camera_parameters)
    gpu, gsegs = _gpu_image(scn, cam, W, H, samps, count_segments=True)
    sp, ca = _oracle_scene(scn, cam)
    ref, rsegs = po.render_xs_f32(sp, ca, W, H, samps, 2, SEED)
    _check_equal(gpu, ref)
    assert gsegs == rsegs
    nseg, ntest, nbox = _gpu_image.tests
    n = len(scn.spheres)
    if n <= 64:
        # linear scan: the tests each lane executed (box mode: about one wall
        # and the three small spheres per segment), of them nbox wall tests
        assert nseg <= ntest <= nseg * n and nbox <= ntest
        if name == "simple":  # no wall pairs, no box mode: every sphere per segment
            assert ntest == nseg * n
        if name in ("box", "box_mirror"):  # box mode: 3 small spheres + >= 1 wall per segment
            assert ntest - nbox == 3 * nseg and nseg <= nbox < 1.5 * nseg
    else:  # BVH: far fewer sphere tests than the linear scan
        assert 0 < ntest < nseg * n / 5 and nbox > 0


def test_wide_bvh_overflow_scene_bitexact():
    """An overlap-heavy cluster (tests/wide_scenes.py): 87 % of the rays
    overflow the wide walk's two-entry stack (tools/wide_stack_depth.cpp), so
    the continuation fallback runs constantly; the image stays bit-exact with
    the oracle's linear scan."""
    _require_gpu()
    from wide_scenes import cluster_scene
    W, H, samps = 48, 27, 4
    scn = cluster_scene(1500, W, H)
    cam = ptgpu.camera.with_config(scn.camera_parameters)
    gpu, gsegs = _gpu_image(scn, cam, W, H, samps, count_segments=True)
    sp, ca = _oracle_scene(scn, cam)
    ref, rsegs = po.render_xs_f32(sp, ca, W, H, samps, 2, SEED)
    _check_equal(gpu, ref)
    assert gsegs == rsegs
    assert float(ref.mean()) > 0.01  # the cluster is in view and lit


@pytest.mark.parametrize("n_small", [0, 1, 4])
def test_wide_bvh_empty_and_one_leaf_trees(n_small):
    """> 64 spheres, nearly all huge: the BVH path with an empty tree (every
    sphere tested linearly) or a tree that is a single leaf (one wide node
    with one child and three empty slots) -- bit-exact with the oracle."""
    _require_gpu()
    from wide_scenes import huge_only_scene
    W, H, samps = 40, 30, 4
    scn = huge_only_scene(70, n_small, W, H)
    assert len(scn.spheres) > 64
    cam = ptgpu.camera.with_config(scn.camera_parameters)
    gpu, gsegs = _gpu_image(scn, cam, W, H, samps, count_segments=True)
    sp, ca = _oracle_scene(scn, cam)
    ref, rsegs = po.render_xs_f32(sp, ca, W, H, samps, 2, SEED)
    _check_equal(gpu, ref)
    assert gsegs == rsegs
    assert float(ref.mean()) > 0.0


@pytest.mark.parametrize("order", [[5, 6, 7, 0, 1, 2, 3, 4], [0, 5, 1, 6, 2, 7, 3, 4], [7, 6, 5, 4, 3, 2, 1, 0]])
def test_sphere_order_layouts(order):
    """The host regroups the records into scan order (axis-anchored walls by
    axis, other huge spheres, small spheres); whatever order the scene lists
    its spheres in, the image stays bit-exact with the oracle, which visits
    them in the same scan order."""
    _require_gpu()
    W, H, samps = 48, 32, 8
    scn = ptgpu.make_scene("box_mirror", W, H)
    scn.spheres = [scn.spheres[i] for i in order]
    cam = ptgpu.camera.with_config(scn.camera_parameters)
    gpu, gsegs = _gpu_image(scn, cam, W, H, samps, count_segments=True)
    sp, ca = _oracle_scene(scn, cam)
    ref, rsegs = po.render_xs_f32(sp, ca, W, H, samps, 2, SEED)
    _check_equal(gpu, ref)
    assert gsegs == rsegs


def test_tilted_huge_spheres_take_the_general_anchor():
    """Huge spheres whose camera-facing point is far from every axis point
    (a 45-degree wall) keep the general anchored form; mixed with the axis
    walls and listed after small spheres, the image stays bit-exact."""
    _require_gpu()
    W, H, samps = 48, 32, 8
    scn = ptgpu.make_scene("box", W, H)
    R = 1e6
    k = R / 2 ** 0.5
    tilted = ptgpu.sphere(R, (k + 0.3, 0.0, -k - 0.3), (0.0, 0.0, 0.0), (0.2, 0.6, 0.6),
                          ptgpu.reflection_type.specular)
    scn.spheres = scn.spheres[5:] + [tilted] + scn.spheres[:5]
    cam = ptgpu.camera.with_config(scn.camera_parameters)
    gpu, gsegs = _gpu_image(scn, cam, W, H, samps, count_segments=True)
    sp, ca = _oracle_scene(scn, cam)
    ref, rsegs = po.render_xs_f32(sp, ca, W, H, samps, 2, SEED)
    _check_equal(gpu, ref)
    assert gsegs == rsegs
    # x and y walls form wall pairs (3 + axis); the back wall (z) is unpaired
    assert po.anchor_axes(sp, ca) == [-1, -1, -1, -1, 3, 3, 2, 4, 4]


@pytest.mark.parametrize("cam_pos", [(0.6, 0.0, 2.0), (0.0, -0.55, 0.3), (0.3, 0.2, 40.0)])
def test_wall_pairs_with_origins_outside_the_room(cam_pos):
    """Wall pairs: a lane whose origin lies outside the room (here the camera
    beyond the right wall, below the floor, or far in front of the open box)
    tests both walls of a pair; the image stays bit-exact with the oracle."""
    _require_gpu()
    W, H, samps = 48, 32, 8
    scn = ptgpu.make_scene("box", W, H)
    scn.camera_parameters.position = cam_pos
    cam = ptgpu.camera.with_config(scn.camera_parameters)
    gpu, gsegs = _gpu_image(scn, cam, W, H, samps, count_segments=True)
    sp, ca = _oracle_scene(scn, cam)
    ref, rsegs = po.render_xs_f32(sp, ca, W, H, samps, 2, SEED)
    _check_equal(gpu, ref)
    assert gsegs == rsegs


@pytest.mark.parametrize("variant", ["crossed", "double_right", "no_left"])
def test_wall_pair_degenerate_layouts(variant):
    """Wall pairs in odd rooms: crossed walls (the - wall's plane beyond the +
    wall's: every origin counts as outside, both walls tested), a second
    right wall (unpaired, tested by every ray after the pair), no left wall
    (no x pair).  Bit-exact with the oracle, and the library's layout equals
    the oracle's."""
    _require_gpu()
    W, H, samps = 48, 32, 8
    scn = ptgpu.make_scene("box", W, H)
    R = 1e6
    if variant == "crossed":
        scn.spheres[0] = ptgpu.sphere(R, (-R + 0.5, 0.0, -1.0), (0.0, 0.0, 0.0), (0.9, 0.1, 0.2),
                                      ptgpu.reflection_type.diffuse)
    elif variant == "double_right":
        scn.spheres.append(ptgpu.sphere(R, (R + 0.3, 0.0, -1.0), (0.0, 0.0, 0.0), (0.2, 0.8, 0.8),
                                        ptgpu.reflection_type.specular))
    else:
        scn.spheres = scn.spheres[1:]
    cam = ptgpu.camera.with_config(scn.camera_parameters)
    sp, ca = _oracle_scene(scn, cam)
    assert ptgpu.scene_layout(scn, cam) == po.scan_layout(sp, ca)
    gpu, gsegs = _gpu_image(scn, cam, W, H, samps, count_segments=True)
    ref, rsegs = po.render_xs_f32(sp, ca, W, H, samps, 2, SEED)
    _check_equal(gpu, ref)
    assert gsegs == rsegs


@pytest.mark.parametrize("name", ["box", "box_mirror", "simple", "synthetic:300", "synthetic:3000"])
def test_per_path_radiance_bitexact(name):
    _require_gpu()
    W, H = 160, 120
    scn = ptgpu.make_scene(name, W, H)
    cam = ptgpu.camera.with_config(scn.camera_parameters)
    rng = np.random.default_rng(7)
    n = 1500
    coords = np.stack([rng.integers(0, W, n), rng.integers(0, H, n), rng.integers(0, 2, n),
                       rng.integers(0, 2, n), rng.integers(0, 1 << 20, n)], axis=1).astype(np.int32)
    p = ptgpu.make_params(W, H, 1, 2, SEED, flags=EXACT)
    with ptgpu.Context(scn, cam) as ctx:
        out, segs = ctx.trace_samples(torch.from_numpy(coords).cuda(), p)
    out = out.cpu().numpy()
    segs = segs.cpu().numpy()
    sp, ca = _oracle_scene(scn, cam)
    for i in range(n):
        x, y, sx, sy, s = (int(v) for v in coords[i])
        ref, rs = po.sample_f32(sp, ca, W, H, 2, SEED, x, y, sx, sy, s)
        assert segs[i] == rs, (i, coords[i])
        assert out[i].tobytes() == ref.tobytes(), (i, coords[i], out[i], ref)


@pytest.mark.parametrize("chunk", [1, 3, 7, 16])
def test_work_unit_size_does_not_change_a_bit(chunk):
    """The exact (u64) sample accumulation makes the image independent of how
    the samples are split into work units (and of lane scheduling)."""
    _require_gpu()
    W, H, samps = 40, 24, 16
    scn = ptgpu.box_mirror_scene(W, H)
    cam = ptgpu.camera.with_config(scn.camera_parameters)
    gpu, gsegs = _gpu_image(scn, cam, W, H, samps, chunk=chunk, count_segments=True)
    sp, ca = _oracle_scene(scn, cam)
    ref, rsegs = po.render_xs_f32(sp, ca, W, H, samps, 2, SEED)
    _check_equal(gpu, ref)
    assert gsegs == rsegs


@pytest.mark.parametrize("nsub", [1, 3])
def test_other_subpixel_counts(nsub):
    _require_gpu()
    W, H = 37, 23  # ragged: not a multiple of the 16-pixel wave width
    scn = ptgpu.box_scene(W, H)
    cam = ptgpu.camera.with_config(scn.camera_parameters)
    gpu, _ = _gpu_image(scn, cam, W, H, 8, nsub=nsub)
    sp, ca = _oracle_scene(scn, cam)
    ref, _ = po.render_xs_f32(sp, ca, W, H, 8, nsub, SEED)
    _check_equal(gpu, ref)


def test_zero_samples_and_tiny_images():
    _require_gpu()
    for W, H in [(1, 1), (17, 3)]:
        scn = ptgpu.box_scene(W, H)
        cam = ptgpu.camera.with_config(scn.camera_parameters)
        gpu, _ = _gpu_image(scn, cam, W, H, 0)
        assert (gpu == 0).all()  # main.cpp:184 loop runs 0 times -> clamp(0) = 0
        gpu, _ = _gpu_image(scn, cam, W, H, 4)
        sp, ca = _oracle_scene(scn, cam)
        ref, _ = po.render_xs_f32(sp, ca, W, H, 4, 2, SEED)
        _check_equal(gpu, ref)


def test_drop_in_render_adds_into_double_image():
    _require_gpu()
    W, H, samps = 48, 32, 8
    scn = ptgpu.box_mirror_scene(W, H)
    cam = ptgpu.camera.with_config(scn.camera_parameters)
    img = np.zeros((H * W, 3), dtype=np.float64)
    ptgpu.render(scn, cam, img, W, H, samps, flags=EXACT)
    sp, ca = _oracle_scene(scn, cam)
    ref, _ = po.render_xs_f32(sp, ca, W, H, samps, 2, SEED)
    assert np.array_equal(img.reshape(H, W, 3), ref.astype(np.float64))
    ptgpu.render(scn, cam, img, W, H, samps, flags=EXACT)  # accumulates like image[row] += (main.cpp:196)
    assert np.array_equal(img.reshape(H, W, 3), 2.0 * ref.astype(np.float64))


def test_shard_invariance_full_size():
    """Tile sharding does not change a single bit (RNG keyed by global pixel):
    at the bench resolution, the 4 interleaved-band slabs of a 4-way shard,
    unsharded on the device, equal the 1-GPU image."""
    _require_gpu()
    W, H, samps = 1920, 1080, 2
    scn = ptgpu.box_scene(W, H)
    cam = ptgpu.camera.with_config(scn.camera_parameters)
    full, _ = _gpu_image(scn, cam, W, H, samps)
    count, br = 4, 8
    rows = ptgpu.shard_rows(H, br, count)
    gathered = torch.zeros((count, rows * W * 3), dtype=torch.float32, device="cuda")
    with ptgpu.Context(scn, cam) as ctx:
        for k in range(count):
            ctx.render_device(gathered[k], ptgpu.make_params(W, H, samps, 2, SEED, br, k, count, flags=EXACT))
        image = torch.empty((H, W, 3), dtype=torch.float32, device="cuda")
        ptgpu.unshard_device(gathered, image, W, H, br, count)
        torch.cuda.synchronize()
    assert np.array_equal(image.cpu().numpy(), full[:H])
    # host statement of the same permutation
    assert np.array_equal(ptgpu.unshard_host(gathered.cpu().numpy(), W, H, br, count), full[:H])
    assert full.min() >= 0.0 and full.max() <= 1.0
    # a bounded oracle check at full size: every 97th row
    sp, ca = _oracle_scene(scn, cam)
    ref, _ = po.render_xs_f32(sp, ca, W, H, samps, 2, SEED, rows=(0, H, 97))
    ys = np.arange(0, H, 97)
    _check_equal(full[H - 1 - ys], ref[H - 1 - ys])


def test_determinism_and_seed_dependence():
    _require_gpu()
    W, H = 64, 48
    scn = ptgpu.box_scene(W, H)
    cam = ptgpu.camera.with_config(scn.camera_parameters)
    a, _ = _gpu_image(scn, cam, W, H, 8)
    b, _ = _gpu_image(scn, cam, W, H, 8)
    c, _ = _gpu_image(scn, cam, W, H, 8, seed=SEED + 1)
    assert np.array_equal(a, b)
    assert not np.array_equal(a, c)


def test_tonemap_matches_reference_formula():
    _require_gpu()
    x = np.concatenate([np.linspace(-0.5, 1.5, 4001), np.random.default_rng(3).random(4000)]).astype(np.float32)
    d = torch.from_numpy(x).cuda()
    out = torch.empty(x.size, dtype=torch.uint8, device="cuda")
    ptgpu.tonemap_device(d, out)
    torch.cuda.synchronize()
    ref = po.tonemap(x.astype(np.float64))
    assert np.array_equal(out.cpu().numpy().astype(np.int32), ref)


def test_invalid_arguments_fail_loudly():
    _require_gpu()
    scn = ptgpu.box_scene(8, 8)
    cam = ptgpu.camera.with_config(scn.camera_parameters)
    img = np.zeros((64, 3))
    with pytest.raises(ptgpu.PtgError):
        ptgpu.render(scn, cam, img, 8, 8, 4, num_subpixels=9, flags=EXACT)
    with pytest.raises(ptgpu.PtgError):
        ptgpu.render(scn, cam, img, 8, 8, -1, flags=EXACT)


def test_progressive_accumulation_matches_one_shot():
    """f2 (README.md:9): sample passes into the exact accumulator; a preview
    after k samples equals a k-sample render, the last resolve equals the
    one-shot frame bit for bit."""
    _require_gpu()
    W, H, samps = 40, 24, 16
    scn = ptgpu.box_scene(W, H)
    cam = ptgpu.camera.with_config(scn.camera_parameters)
    p = ptgpu.make_params(W, H, samps, 2, SEED, flags=EXACT)
    rows = ptgpu.shard_rows(H, 8, 1)
    out = torch.empty(rows * W * 3, dtype=torch.float32, device="cuda")
    sp, ca = _oracle_scene(scn, cam)
    with ptgpu.Context(scn, cam) as ctx:
        ctx.reset_accumulation(p)
        done = 0
        for end in (3, 10, 16):
            ctx.accumulate(p, done, end)
            done = end
            ctx.resolve(out, p, done)
            torch.cuda.synchronize()
            img = out.cpu().numpy().reshape(rows, W, 3)[:H]
            ref, _ = po.render_xs_f32(sp, ca, W, H, done, 2, SEED)
            _check_equal(img, ref)
        one, _ = _gpu_image(scn, cam, W, H, samps)
        assert np.array_equal(img, one)


def test_scene_file_renders_like_the_builtin_scene(tmp_path):
    """f4: a scene written to a file and read back renders the same bits."""
    _require_gpu()
    W, H, samps = 48, 32, 8
    scn = ptgpu.box_mirror_scene(W, H)
    path = tmp_path / "mirror.scene"
    ptgpu.save_scene_file(scn, str(path))
    back = ptgpu.make_scene(str(path), W, H)
    a, _ = _gpu_image(scn, ptgpu.camera.with_config(scn.camera_parameters), W, H, samps)
    b, _ = _gpu_image(back, ptgpu.camera.with_config(back.camera_parameters), W, H, samps)
    assert np.array_equal(a, b)


def test_cli_renders_and_splits_over_devices(tmp_path):
    """The C++ CLI (host/main.cpp): by default the drop-in ptg_render; with
    --devices the single-process multi-GPU path ptg_render_multi (shards +
    ONE RCCL gather) -- on this one-GPU box a one-rank communicator, whose
    P6 bytes equal the default's; a repeated device is refused (RCCL needs
    one rank per GPU).  The bytes are the reference's color_to_int of the
    drop-in image (utils.cpp:11-16)."""
    _require_gpu()
    import os
    import subprocess
    cli = os.path.join(os.path.dirname(ptgpu.LIB_PATH), "pt_render_gpu")
    W, H, spp = 40, 30, 16
    outs = {}
    for devs in (None, "0"):
        out = tmp_path / f"img_{devs}.ppm"
        cmd = [cli, "--scene", "box", "--width", str(W), "--height", str(H), "--spp", str(spp), "--format", "p6",
               "--out", str(out)] + (["--devices", devs] if devs else [])
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, r.stderr
        outs[devs] = out.read_bytes()
    assert outs[None] == outs["0"]
    r = subprocess.run([cli, "--scene", "box", "--width", str(W), "--height", str(H), "--devices", "0,0",
                        "--out", str(tmp_path / "dup.ppm")], capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "distinct devices" in r.stderr
    outs["0"] = outs[None]
    header = f"P6\n{W} {H}\n255\n".encode()
    assert outs["0"].startswith(header)
    scn = ptgpu.box_scene(W, H)
    img = np.zeros((H * W, 3))
    ptgpu.render(scn, ptgpu.camera.with_config(scn.camera_parameters), img, W, H, spp // 4)  # the CLI's default mode
    ref = po.tonemap(img).astype(np.uint8).tobytes()
    assert outs["0"][len(header):] == ref
    # --exact-math: the bytes of the CPU oracle's image (Mode B, color_to_int)
    out = tmp_path / "img_exact.ppm"
    r = subprocess.run([cli, "--scene", "box", "--width", str(W), "--height", str(H), "--spp", str(spp), "--format",
                        "p6", "--exact-math", "--out", str(out)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    sp, ca = _oracle_scene(scn, ptgpu.camera.with_config(scn.camera_parameters))
    b, _ = po.render_xs_f32(sp, ca, W, H, spp // 4, 2, ptgpu.DEFAULT_SEED)
    assert out.read_bytes()[len(header):] == po.tonemap(b.astype(np.float64)).astype(np.uint8).tobytes()


def test_split_tail_frame_is_exact():
    """A large frame with whole-pixel units runs its last rows as the split
    tail (8 accumulated units per pixel group + resolve_kernel for those rows,
    fill_launch): the image equals the same frame with every pixel group split
    into explicit chunks, and the oracle on rows of both regions."""
    _require_gpu()
    W, H, samps = 1920, 1080, 8
    scn = ptgpu.box_scene(W, H)
    cam = ptgpu.camera.with_config(scn.camera_parameters)
    tail, _ = _gpu_image(scn, cam, W, H, samps, band_rows=1)
    chunked, _ = _gpu_image(scn, cam, W, H, samps, band_rows=1, chunk=3)
    assert np.array_equal(tail, chunked)
    sp, ca = _oracle_scene(scn, cam)
    for y in (0, 1, 2, 537, H - 1):  # y = 0.. are the bottom image rows = the last slab rows (the tail)
        ref, _ = po.render_xs_f32(sp, ca, W, H, samps, 2, SEED, rows=(y, y + 1, 1))
        _check_equal(tail[H - 1 - y], ref[H - 1 - y])


def test_shards_with_split_tail_are_exact():
    """2-, 4- and 8-way shards of a full-size frame run whole-pixel units with
    a split tail (fill_launch: from 1.5 rounds of wave slots on); gathered,
    they equal the 1-GPU frame bit for bit, and rows of the last slab rows
    (the split tail of each shard) equal the oracle."""
    _require_gpu()
    W, H, samps = 1920, 1080, 8
    scn = ptgpu.box_scene(W, H)
    cam = ptgpu.camera.with_config(scn.camera_parameters)
    full, _ = _gpu_image(scn, cam, W, H, samps, band_rows=1)
    sp, ca = _oracle_scene(scn, cam)
    with ptgpu.Context(scn, cam) as ctx:
        for count in (2, 4, 8):
            rows = ptgpu.shard_rows(H, 1, count)
            gathered = torch.zeros((count, rows * W * 3), dtype=torch.float32, device="cuda")
            for k in range(count):
                ctx.render_device(gathered[k], ptgpu.make_params(W, H, samps, 2, SEED, 1, k, count, flags=EXACT))
            image = torch.empty((H, W, 3), dtype=torch.float32, device="cuda")
            ptgpu.unshard_device(gathered, image, W, H, 1, count)
            torch.cuda.synchronize()
            assert np.array_equal(image.cpu().numpy(), full), count
    # image row H-1-y sits in slab row (H-1-y) // count: y = 0, 1 are in the last slab rows
    for y in (0, 1, H - 1):
        ref, _ = po.render_xs_f32(sp, ca, W, H, samps, 2, SEED, rows=(y, y + 1, 1))
        _check_equal(full[H - 1 - y], ref[H - 1 - y])


def test_bvh_two_level_units_are_exact():
    """A BVH frame below the split-tail threshold (fill_launch: e.g. an 8-way
    shard of C5) runs its head rows in chunks of up to PTG_BVH_HEAD_CHUNK
    samples and the last ~half round of rows in the auto chunk: the image
    equals the same frame in explicit small chunks, and the oracle on a head
    row and a tail row."""
    _require_gpu()
    W, H, samps = 1920, 160, 16
    scn = ptgpu.make_scene("synthetic:300", W, H)
    cam = ptgpu.camera.with_config(scn.camera_parameters)
    two, _ = _gpu_image(scn, cam, W, H, samps, band_rows=1)
    chunked, _ = _gpu_image(scn, cam, W, H, samps, band_rows=1, chunk=3)
    assert np.array_equal(two, chunked)
    sp, ca = _oracle_scene(scn, cam)
    for y in (0, H - 1):  # y = 0: the last slab row (tail level); H - 1: the first (head level)
        ref, _ = po.render_xs_f32(sp, ca, W, H, samps, 2, SEED, rows=(y, y + 1, 1))
        _check_equal(two[H - 1 - y], ref[H - 1 - y])


def test_render_multi_rccl_one_rank_is_exact():
    """ptg_render_multi (ncclCommInitAll + ONE ncclGather +
    un-shard) executes on hardware here as a one-rank communicator: the
    image equals the drop-in ptg_render's bit for bit for several band
    heights; repeated devices are refused."""
    _require_gpu()
    W, H, samps = 52, 30, 8
    scn = ptgpu.box_mirror_scene(W, H)
    cam = ptgpu.camera.with_config(scn.camera_parameters)
    ref = np.zeros((H * W, 3))
    ptgpu.render(scn, cam, ref, W, H, samps, flags=EXACT)
    # each call is a fresh context on a non-blocking stream (its first frame
    # once raced a null-stream zeroing of the accumulator: ensure_acc)
    for br in (1, 4, 2, 8, 4):
        img = np.zeros((H * W, 3))
        ptgpu.render_multi(scn, cam, img, W, H, samps, [0], band_rows=br, flags=EXACT)
        assert np.array_equal(img, ref), br
    with pytest.raises(ptgpu.PtgError, match="distinct devices"):
        ptgpu.render_multi(scn, cam, np.zeros((H * W, 3)), W, H, samps, [0, 0])


def test_render_sharded_on_nccl_backend():
    """render_sharded (the multi-process path) on the nccl backend -- RCCL --
    at world size 1: the gathered, un-sharded image equals the one-GPU
    frame bit for bit (the 8-GPU run is the driver's)."""
    _require_gpu()
    import socket

    import torch.distributed as dist
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    W, H, samps = 48, 32, 8
    scn = ptgpu.box_scene(W, H)
    cam = ptgpu.camera.with_config(scn.camera_parameters)
    full, _ = _gpu_image(scn, cam, W, H, samps, band_rows=1)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    try:
        assert dist.get_backend() == "nccl"
        p = ptgpu.make_params(W, H, samps, 2, SEED, 1, 0, 1, flags=EXACT)
        slab = torch.zeros(ptgpu.shard_rows(H, 1, 1) * W * 3, dtype=torch.float32, device="cuda")
        with ptgpu.Context(scn, cam) as ctx:
            image = ptgpu.render_sharded(p, slab, ctx=ctx)
            torch.cuda.synchronize()
        assert np.array_equal(image.cpu().numpy(), full)
    finally:
        dist.destroy_process_group()


def test_c4_frame_size_shards_are_exact():
    """C4's frame size (box 3840x2160, BASELINE configs[3], at 8 spp here):
    the 1-GPU frame, its 8-way interleaved shards gathered and un-sharded on
    the device, and oracle rows (head and split-tail rows) agree bit for
    bit."""
    _require_gpu()
    W, H, samps = 3840, 2160, 2
    scn = ptgpu.box_scene(W, H)
    cam = ptgpu.camera.with_config(scn.camera_parameters)
    full, _ = _gpu_image(scn, cam, W, H, samps, band_rows=1)
    count = 8
    rows = ptgpu.shard_rows(H, 1, count)
    gathered = torch.zeros((count, rows * W * 3), dtype=torch.float32, device="cuda")
    with ptgpu.Context(scn, cam) as ctx:
        for k in range(count):
            ctx.render_device(gathered[k], ptgpu.make_params(W, H, samps, 2, SEED, 1, k, count, flags=EXACT))
        image = torch.empty((H, W, 3), dtype=torch.float32, device="cuda")
        ptgpu.unshard_device(gathered, image, W, H, 1, count)
        torch.cuda.synchronize()
    assert np.array_equal(image.cpu().numpy(), full)
    sp, ca = _oracle_scene(scn, cam)
    for y in (0, 1, 1337, H - 1):
        ref, _ = po.render_xs_f32(sp, ca, W, H, samps, 2, SEED, rows=(y, y + 1, 1))
        _check_equal(full[H - 1 - y], ref[H - 1 - y])


def test_c5_frame_size_rows_are_exact():
    """C5's frame size (synthetic:10000 at 1920x1080, BVH kernel with
    whole-pixel units and a split tail, at 64 spp here): rows of the head
    and of the tail equal the oracle's linear scan bit for bit."""
    _require_gpu()
    W, H, samps = 1920, 1080, 16
    scn = ptgpu.make_scene("synthetic:10000", W, H)
    cam = ptgpu.camera.with_config(scn.camera_parameters)
    full, _ = _gpu_image(scn, cam, W, H, samps, band_rows=1)
    sp, ca = _oracle_scene(scn, cam)
    for y in (0, 300):  # y = 0: the last slab row (split tail); 300: a head row in the sphere field
        ref, _ = po.render_xs_f32(sp, ca, W, H, samps, 2, SEED, rows=(y, y + 1, 1), nthreads=16)
        _check_equal(full[H - 1 - y], ref[H - 1 - y])


@pytest.mark.parametrize("samps", [8, 37])
def test_bvh_pixel_split_tail_is_exact(samps):
    """The BVH kernel's split tail (fill_launch, PTG_BVH_TAIL_PSPLIT): the
    last rows (PTG_BVH_TAIL_HALF_ROUNDS half rounds of wave slots) run each
    16-pixel group as 8 units of 2 interleaved pixels (PTG_BVH_TAIL_CHUNKS_MANY
    at this frame's >= 5 rounds, PTG_TAIL_CHUNKS below: both 8) with every
    sample (resolved in the wave, no HBM accumulation) -- the frame
    equals the same frame in explicit sample chunks, and oracle rows of the
    tail (y = 0, 1) and the head equal the oracle's linear scan."""
    _require_gpu()
    W, H = 1920, 1080
    scn = ptgpu.make_scene("synthetic:300", W, H)
    cam = ptgpu.camera.with_config(scn.camera_parameters)
    tail, _ = _gpu_image(scn, cam, W, H, samps, band_rows=1)
    chunked, _ = _gpu_image(scn, cam, W, H, samps, band_rows=1, chunk=3)
    assert np.array_equal(tail, chunked)
    sp, ca = _oracle_scene(scn, cam)
    for y in (0, 1, 700):
        ref, _ = po.render_xs_rect(sp, ca, W, H, samps, 2, SEED, rows=(y, y + 1, 1), nthreads=16)
        _check_equal(tail[H - 1 - y], ref[H - 1 - y])


def test_parameter_limits_refused_cleanly():
    """The boundary's limits (check_params): a frame the kernel's indexing
    does not cover is refused with an error before anything is launched,
    and the context stays usable.  Width >= 2^20 (the slot table packs x in
    20 bits), more than 2^28 pixels, more than 8 sub-pixels per axis, a
    negative sample count and a shard rank outside its count."""
    _require_gpu()
    scn = ptgpu.make_scene("box", 64, 48)
    cam = ptgpu.camera.with_config(scn.camera_parameters)
    bad = [dict(w=1 << 20, h=1), dict(w=1 << 15, h=1 << 14), dict(nsub=9), dict(samps=-1),
           dict(rank=2, count=2), dict(w=0)]
    with ptgpu.Context(scn, cam) as ctx:
        for b in bad:
            p = ptgpu.make_params(b.get("w", 64), b.get("h", 48), b.get("samps", 4), b.get("nsub", 2), SEED, 1,
                                  b.get("rank", 0), b.get("count", 1))
            with pytest.raises(ptgpu.PtgError):
                ctx.launch_info(p)
        # the largest accepted shapes still plan a launch
        for w, h, nsub in ((1 << 20) - 1, 1, 2), (1 << 14, 1 << 14, 8):
            info = ctx.launch_info(ptgpu.make_params(w, h, 4, nsub, SEED))
            assert info["units"] > 0 and info["workgroups"] > 0
        # and the context still renders
        out = torch.empty(48 * 64 * 3, dtype=torch.float32, device="cuda")
        ctx.render_device(out, ptgpu.make_params(64, 48, 4, 2, SEED))
        torch.cuda.synchronize()
        assert float(out.max()) > 0.0
