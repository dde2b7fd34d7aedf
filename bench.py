#!/usr/bin/env python3
"""Benchmark: Mray-samples/s of the MI355X render loop (BASELINE.json metric).

One step = one full frame of the workload rendered by the HIP megakernel,
scene and output already resident in HBM.  Workload: the metric's frame,
box_scene.hpp at 1920x1080, 1024 spp (256 samples per sub-pixel), for EVERY
N -- so the N = 1, 2, 4, 8 lines of a scaling run measure the same frame.
With N > 1 GPUs the frame is tile-sharded by interleaved row bands, the step
including the single gather (RCCL over xGMI) to rank 0 and the un-shard.
value = whole-frame samples / max-over-ranks time (strong scaling: the frame
is fixed).  At N > 1 rank 0 first renders the same frame alone (untimed for
`value`) and the line carries t1_ms and efficiency = T1 / (N * T_N) of this
run, so the scaling line is self-contained.  --workload c1..c5 picks another
BASELINE.json config (C4: box 3840x2160x4096spp); the line's metric string
then names the frame actually rendered.  Every N > 1 line carries what the
RCCL group actually was -- rccl_ranks (ncclCommCount of every communicator),
the devices and their PCI bus ids -- and bench.py exits 3 instead of printing
a line when fewer than N ranks or distinct devices took part.

Launch modes (resolve_launch):
  * WORLD_SIZE unset, --gpus 1           one GPU.
  * WORLD_SIZE unset, --gpus N > 1       ONE process drives GPUs 0..N-1
                                         through ptg_multi (csrc/ptg_multi.cpp):
                                         N shards, ONE ncclGather (RCCL over
                                         xGMI, communicators from
                                         ncclCommInitAll), the un-shard on GPU 0
                                         -- no launcher needed.
  * WORLD_SIZE = N (torchrun)            one process per GPU, torch.distributed
                                         on nccl (RCCL); the gather is
                                         ptgpu.render_sharded's.
  * WORLD_SIZE set and != --gpus         an error (exit 2): the line would
                                         otherwise claim a GPU count it did not
                                         measure.
  * --launch inprocess                   the one-process ptg_multi path at any N,
                                         also N = 1 (a one-rank RCCL group: the
                                         1-GPU box rehearsal of that path).
PTG_REHEARSAL=1 runs either N > 1 mode on one GPU (N shards on device 0; gloo
for torchrun) -- a 1-GPU box rehearsal of the sharded path, labelled as such.
Efficiency = T1 / (N * T_N) with T1 and T_N timed the same way: wall clock
per frame over the same kind of step (render + gather + un-shard), and again
from the kernels' HIP events alone (efficiency_kernel).

Also reported:
  roofline     -- VALU fp32 roofline of the render kernel: algorithmic FLOP
                  per launch (S_bar*(23*N_spheres + 100) + 60 per sample,
                  SURVEY.md 8(d), S_bar measured by the kernel's own segment
                  counter) / its average launch time from HIP events on the
                  launch stream; peak 157.3 TFLOP/s (MI355X fp32 vector, the
                  packed rate) -> frac, and 78.6 TFLOP/s (the non-packed
                  issue rate: the kernel is built without v_pk_*_f32, which on
                  gfx950 cost two plain issue slots, MI355X_MICROARCH.md:491)
                  -> frac_nonpacked; valu_fp32_share = FP32 add/mul/fma/trans
                  instructions / all VALU instructions of the committed
                  rocprofv3 profile of the workload.
  cpu_baseline -- the REFERENCE's own per-pixel code (src/main.cpp:27-197
                  compiled with its `pt` library into oracle/_ref/libref_main.so,
                  kind "reference") in an OpenMP row loop on the host's cores,
                  on a bounded sample of the same workload, rank 0 at N=1 only;
                  beside it the repo's C restatement (oracle Mode A, "port") on
                  the same sample, and the quality rows of the benchmarked frame
                  against the oracle.

Arithmetic: the default (product) mode takes square roots, reciprocal
square roots, the hit division and sin/cos from the GPU's transcendental
instructions; --exact-math renders with PTG_FLAG_EXACT_MATH (bit for bit the
oracle's Mode B).  Both are fp32; config.arithmetic names the mode.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "cpu-path-tracing_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import ptgpu  # noqa: E402

METRIC = "Mray-samples/sec at 1920×1080×1024spp; per-pixel RMSE vs CPU ref"
PEAK_FP32_TFLOPS = 157.3  # MI355X_MICROARCH.md: peak FP32 vector (= f32 MFMA) rate, packed
# the non-packed FP32 VALU rate (256 CUs x 4 SIMDs x 32 lanes x 2 FLOP x 2.4
# GHz): what a kernel without v_pk_*_f32 can issue at most
PEAK_FP32_NONPACKED_TFLOPS = 78.6


# BASELINE.json configs (C1..C5) plus the metric's own frame
# (the default workload at every N)
WORKLOADS = {
    "bench": ("box", 1920, 1080, 1024),       # the metric: box_scene at 1920x1080x1024spp on one MI355X
    "c1": ("simple", 400, 300, 64),
    "c2": ("box", 1024, 768, 256),
    "c3": ("box_mirror", 1920, 1080, 1024),
    "c4": ("box", 3840, 2160, 4096),          # tile-sharded over 8 GPUs
    "c5": ("synthetic:10000", 1920, 1080, 1024),
}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def host_cpu_info():
    """The host the CPU baseline runs on: the machine's CPU count and model,
    the CPUs this process may run on, the cgroup CPU quota and
    OMP_NUM_THREADS (on the GPU box the job's share of a large machine)."""
    info = {"nproc": os.cpu_count()}
    try:
        info["affinity"] = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        pass
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, period = f.read().split()[:2]
            info["cgroup_cpus"] = None if q == "max" else round(int(q) / int(period), 2)
    except (OSError, ValueError):
        pass
    info["omp_num_threads"] = os.environ.get("OMP_NUM_THREADS")
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    info["cpu_model"] = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return info


def default_cpu_threads():
    """Threads for the CPU baseline: the job's CPU share -- OMP_NUM_THREADS
    when set (16 on the GPU box, where os.cpu_count() is the whole machine's
    CPUs shared with other jobs), else the CPUs this process may run on."""
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit() and int(env) > 0:
        return int(env)
    try:
        return len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        return os.cpu_count() or 1


def cpu_baseline(scene_name, W, H, samps, nsub, threads, row_step, gpu_image=None, seed=None, quality_rows=4):
    """Time the reference's own per-pixel code on the host: every row_step-th
    row of the frame, all samples of those rows, in an OpenMP
    schedule(dynamic,1) row loop (main.cpp:217-234's task body, per-row
    mt19937(RD * (unsigned short)(y^3)) with RD = 1 for random_device); the
    rate extrapolates linearly to the frame.  kind "reference" when
    oracle/_ref/libref_main.so was built (the reference compiled in this
    container, shipped with the tree), else the restatement ("port").  The
    port (oracle Mode A: the same algorithm restated in C, same seeds) is
    timed on the same rows beside it.

    With `gpu_image` (the benchmarked frame, [H, W, 3] float32) the same leg
    also checks quality on `quality_rows` evenly spaced rows:
    per-pixel RMSE and max |diff| of the GPU image against the identically
    seeded fp32 CPU restatement (Mode B, the checker: 0 when bit-exact), and
    the RMSE of that against the same path in double arithmetic with the same
    counter RNG (Mode A/xs) -- the effect of computing in fp32; and the GPU
    image's own RMSE against Mode A/xs, the north star's bar (< 1e-3)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    try:
        import pyoracle as po
        po.lib()
    except Exception as e:  # noqa: BLE001
        log(f"cpu_baseline unavailable: {e}")
        return None
    pr = None
    try:
        import pyref
        if pyref.available():
            pyref.lib()
            pr = pyref
        else:
            log("cpu_baseline: oracle/_ref/libref_main.so not built; timing the port only")
    except Exception as e:  # noqa: BLE001
        log(f"cpu_baseline: reference build unusable ({e}); timing the port only")
    scn = ptgpu.make_scene(scene_name, W, H)
    cam = ptgpu.camera.with_config(scn.camera_parameters)
    sp = scn.to_array().view(po.SPHERE_DT)
    ca = cam.to_array().view(po.CAMERA_DT)
    rows = len(range(0, H, row_step))
    nsamp = rows * W * samps * nsub * nsub
    sample = (f"{scene_name} {W}x{H} at {samps * nsub * nsub} spp: every {row_step}th row ({rows} of {H}, all "
              f"their samples) timed, the frame extrapolated linearly; OpenMP schedule(dynamic,1) row loop on "
              f"{threads} threads, per-row mt19937(1 * (unsigned short)(y^3)) (main.cpp:222-223)")

    def timed(fn):
        t0 = time.perf_counter()
        fn()
        return time.perf_counter() - t0

    img = np.zeros(W * H * 3)
    dt_port = timed(lambda: po.lib().po_render_mt(po.ptr(sp), len(sp), po.ptr(ca), W, H, samps, nsub, 1, 0, H,
                                                   row_step, threads, po.ptr(img)))
    port = {"value": round(nsamp / dt_port / 1e6, 4), "seconds": round(dt_port, 2),
            "what": "oracle Mode A (oracle/pt_oracle.c: main.cpp:30-197 restated in C, double + mt19937)"}
    if pr is not None:
        ref_img = np.zeros(W * H * 3)
        seeds = pr.reference_row_seeds(H, 1)
        dt = timed(lambda: pr.render_rows(sp, ca, W, H, samps, nsub, seeds, rows=(0, H, row_step), nthreads=threads,
                                          image=ref_img))
        same = bool(np.array_equal(ref_img, img))
        out = {"value": round(nsamp / dt / 1e6, 4), "unit": "Mray-samples/s", "cores": threads, "kind": "reference",
               "seconds": round(dt, 2), "frame_seconds_extrapolated": round(W * H * samps * nsub * nsub * dt / nsamp, 1),
               "sample": sample + "; the reference's src/main.cpp:27-197 + `pt` library (-O3) via "
                                  "oracle/_ref/libref_main.so",
               "port": dict(port, image_equals_reference=same)}
    else:
        out = {"value": port["value"], "unit": "Mray-samples/s", "cores": threads, "kind": "port",
               "seconds": port["seconds"],
               "frame_seconds_extrapolated": round(W * H * samps * nsub * nsub * dt_port / nsamp, 1),
               "sample": sample + "; " + port["what"]}
    out["host"] = host_cpu_info()
    if gpu_image is not None and quality_rows > 0:
        step_y = max(1, H // quality_rows)
        ys = np.arange(step_y // 2, H, step_y)[:quality_rows]  # image-space y (main.cpp:181: y = 0 at the bottom)
        t1 = time.perf_counter()
        gpu = np.concatenate([gpu_image[H - 1 - y] for y in ys]).astype(np.float64)
        b = np.concatenate([po.render_xs_f32(sp, ca, W, H, samps, nsub, seed, rows=(int(y), int(y) + 1, 1),
                                             nthreads=threads)[0][H - 1 - y] for y in ys]).astype(np.float64)
        a = np.concatenate([po.render_xs_f64(sp, ca, W, H, samps, nsub, seed, rows=(int(y), int(y) + 1, 1),
                                             nthreads=threads)[0][H - 1 - y] for y in ys])
        out["quality"] = {
            "rows": [int(y) for y in ys],
            "rmse_vs_cpu_fp32": float(np.sqrt(((gpu - b) ** 2).mean())),
            "max_abs_vs_cpu_fp32": float(np.abs(gpu - b).max()),
            "rmse_fp32_vs_fp64_same_rng": float(np.sqrt(((b - a) ** 2).mean())),
            "rmse_vs_cpu_fp64_same_rng": float(np.sqrt(((gpu - a) ** 2).mean())),
            "image_mean": float(gpu.mean()),
            "seconds": round(time.perf_counter() - t1, 2),
            "checker": "oracle Mode B (fp32 restatement) / Mode A-xs (double, same counter RNG)"}
    return out


def resolve_launch(gpus, env):
    """(mode, world, rank, local) for --gpus and the launcher's environment:
    "single" (one GPU), "inprocess" (no launcher, --gpus N > 1: one process,
    ptg_multi over GPUs 0..N-1) or "torchrun" (WORLD_SIZE ranks).  A
    WORLD_SIZE that disagrees with --gpus raises ValueError."""
    if gpus < 1:
        raise ValueError(f"--gpus must be >= 1 (got {gpus})")
    ws = env.get("WORLD_SIZE")
    if ws is None or ws == "":
        return ("inprocess" if gpus > 1 else "single"), 1, 0, 0
    world = int(ws)
    if world != gpus:
        raise ValueError(f"--gpus {gpus} but the launcher started WORLD_SIZE={world} ranks: the line would "
                         f"report a GPU count it did not measure")
    rank = int(env.get("RANK", "0"))
    local = int(env.get("LOCAL_RANK", "0"))
    return ("torchrun" if world > 1 else "single"), world, rank, local


def load_pmc(workload):
    """PMC figures of the committed rocprofv3 profile of this workload
    (profiles/pmc_traffic.json, written by profiles/summarize.py): HBM bytes
    per launch (FETCH_SIZE x2 + WRITE_SIZE, MI355X_MICROARCH.md HBM section)
    and the VALU issue utilisation."""
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(p) as f:
            d = json.load(f)
        if d.get("workload") == workload:  # single-record file
            return d
        return d.get(workload, {})
    except (OSError, ValueError):
        pass
    return {}


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--workload", choices=["auto"] + sorted(WORKLOADS), default="auto",
                    help="BASELINE.json config (auto = bench: the metric's box 1920x1080x1024spp frame, at every N; "
                         "c4: box 3840x2160x4096spp)")
    ap.add_argument("--launch", choices=["auto", "inprocess"], default="auto",
                    help="inprocess: the one-process ptg_multi path (RCCL communicators from ncclCommInitAll) "
                         "even at --gpus 1")
    ap.add_argument("--scene", default=None, help="overrides the workload's scene")
    ap.add_argument("--width", type=int, default=None)
    ap.add_argument("--height", type=int, default=None)
    ap.add_argument("--spp", type=int, default=None, help="total samples per pixel (4 sub-pixels)")
    ap.add_argument("--band-rows", type=int, default=ptgpu.DEFAULT_BAND_ROWS)
    ap.add_argument("--chunk", type=int, default=0, help="samples per sub-pixel per work unit (0 = auto)")
    ap.add_argument("--cpu-baseline", choices=["auto", "off"], default="auto")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="CPU baseline threads (0 = the job's CPU share: OMP_NUM_THREADS, else the affinity mask)")
    ap.add_argument("--cpu-row-step", type=int, default=16,
                    help="CPU baseline: time every k-th row of the frame (16 = one sixteenth)")
    ap.add_argument("--exact-math", action="store_true",
                    help="PTG_FLAG_EXACT_MATH: the exact fp32 sequences (bit for bit the CPU oracle's Mode B)")
    ap.add_argument("--reference-f64", action="store_true",
                    help="PTG_FLAG_REFERENCE_F64: the reference's double arithmetic (parity mode, not the metric)")
    ap.add_argument("--t1", choices=["auto", "off"], default="auto",
                    help="N > 1: time the same frame on one GPU first (t1_ms, efficiency)")
    ap.add_argument("--t1-steps", type=int, default=3, help="N > 1: frames timed for T1 (after one warm-up)")
    ap.add_argument("--quality-rows", type=int, default=4,
                    help="rows checked against the CPU oracle in the cpu_baseline leg (0 = none)")
    return ap.parse_args(argv)


def frame_config(args, world):
    """The frame for every N: the metric's (bench) unless --workload / the
    size flags say otherwise (`world` does not change it: a scaling run's
    lines compare one frame)."""
    del world
    wl = args.workload if args.workload != "auto" else "bench"
    wscene, wW, wH, wspp = WORKLOADS[wl]
    scene = args.scene or wscene
    nsub = 2  # main.cpp:202
    W, H = args.width or wW, args.height or wH
    samps = (args.spp or wspp) // (nsub * nsub)  # main.cpp:206
    spp = samps * nsub * nsub
    wl_name = wl if (scene, W, H, spp) == WORKLOADS[wl] else "custom"
    return wl_name, scene, W, H, samps, nsub, spp


def metric_of(scene, W, H, spp):
    """BASELINE.json's metric string when the frame is the metric's own
    (box 1920x1080x1024spp), else the same metric named for the frame
    actually rendered."""
    if (scene, W, H, spp) == WORKLOADS["bench"]:
        return METRIC
    return f"Mray-samples/sec at {W}×{H}×{spp}spp ({scene}); per-pixel RMSE vs CPU ref"


def check_group(n, ranks, devices, bus_ids, rehearsal):
    """Problems with an N-GPU measurement's RCCL group (empty: none): every
    communicator has N ranks, the N ranks run on N distinct devices with N
    distinct PCI bus ids.  A rehearsal (N shards on one GPU) is exempt; None
    entries (not determinable) are not counted as evidence either way."""
    if rehearsal or n <= 1:
        return []
    bad = []
    known = [r for r in ranks if r is not None]
    if any(r != n for r in known):
        bad.append(f"RCCL communicators of {sorted(set(known))} ranks, not {n}")
    kd = [d for d in devices if d is not None and d != ""]
    if len(kd) == n and len(set(kd)) != n:
        bad.append(f"{len(set(kd))} distinct devices for {n} ranks: {devices}")
    kb = [b for b in bus_ids if b]
    if len(kb) == n and len(set(kb)) != n:
        bad.append(f"{len(set(kb))} distinct PCI bus ids for {n} ranks: {bus_ids}")
    return bad


def torch_rccl_info(local):
    """(ncclCommCount, ncclCommCuDevice, ncclCommUserRank) of the default
    process group's RCCL communicator on this rank's device, read with the
    RCCL library torch itself loaded (torch/lib/librccl.so, whose struct the
    handle belongs to); (None, None, None, reason) when not determinable."""
    import ctypes as C
    try:
        pg = dist.distributed_c10d._get_default_group()
        backend = pg._get_backend(torch.device("cuda", local))
        ptr = int(backend._comm_ptr())
        if not ptr:
            return None, None, None, "no communicator"
        path = os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so")
        L = C.CDLL(path if os.path.exists(path) else "librccl.so")
        out = []
        for fn in ("ncclCommCount", "ncclCommCuDevice", "ncclCommUserRank"):
            v = C.c_int(-1)
            rc = getattr(L, fn)(C.c_void_p(ptr), C.byref(v))
            if rc != 0:
                return None, None, None, f"{fn} returned {rc}"
            out.append(int(v.value))
        return out[0], out[1], out[2], None
    except Exception as e:  # noqa: BLE001 -- reported in the line, not fatal
        return None, None, None, f"{type(e).__name__}: {e}"


def bus_id_of(device):
    """PCI bus id of a visible device (hipDeviceGetPCIBusId via the C ABI);
    None when it cannot be read -- not evidence either way in check_group
    (a shared 'unknown' string would read as one bus id for every rank)."""
    try:
        return ptgpu.pci_bus_id(device) or None
    except Exception as e:  # noqa: BLE001
        log(f"warning: PCI bus id of device {device} not readable: {e}")
        return None


def arith_flags(args):
    return (ptgpu.FLAG_REFERENCE_F64 if args.reference_f64 else 0) | (ptgpu.FLAG_EXACT_MATH if args.exact_math else 0)


def arith_name(args):
    return ("reference f64" if args.reference_f64 else
            "exact (PTG_FLAG_EXACT_MATH)" if args.exact_math else
            "fast (hardware v_sqrt/v_rsq/v_rcp/v_sin/v_cos)")


def roofline(frame_samples, seg_total, sph_total, box_total, my_samples, kern_ms, n_sph, pmc):
    """S_bar*(23*N + 100) + 60 FLOP per sample for the linear
    scan (the model: every sphere tested per segment); generalised to the
    tests actually executed for BVH scenes: 23 FLOP per ray-sphere test, 12
    per slab box test, 100 per segment, 60 per sample.  `frac` prices the
    model (the survey's definition); `frac_executed` prices only the tests the
    kernel ran, from its own counters (linear scenes: box mode tests about
    one wall and the three small spheres per segment, not all N spheres; BVH
    scenes: the same as `frac`).  `achieved` is one GPU's kernel: its samples
    x FLOP/sample / its kernel time (HIP events on the launch stream)."""
    linear = n_sph <= 64
    s_bar = seg_total / frame_samples
    exec_tests = sph_total / frame_samples  # sphere tests executed per sample (counting kernel)
    model_tests = s_bar * n_sph if linear else exec_tests
    boxes = 0.0 if linear else box_total / frame_samples  # BVH box tests per sample
    walls = box_total / frame_samples if linear else None  # linear: wall tests executed per sample
    flop_per_sample = 23 * model_tests + 12 * boxes + 100 * s_bar + 60
    flop_exec = 23 * exec_tests + 12 * boxes + 100 * s_bar + 60
    tf = (lambda f: my_samples * f / (kern_ms / 1e3) / 1e12) if kern_ms > 0 else (lambda f: None)
    achieved, achieved_exec = tf(flop_per_sample), tf(flop_exec)
    per_seg = (lambda x: round(x / s_bar, 3) if (s_bar and x is not None) else None)
    out = {
        "bound": "valu", "achieved": round(achieved, 3) if achieved else None,
        "peak": PEAK_FP32_TFLOPS, "unit": "TFLOP/s",
        "frac": round(achieved / PEAK_FP32_TFLOPS, 4) if achieved else None,
        # against the non-packed FP32 issue rate (the kernel is built without
        # v_pk_*_f32: on gfx950 a packed op costs two plain issue slots,
        # MI355X_MICROARCH.md:491, and the pair moves made it 7.8 % slower)
        "peak_nonpacked": PEAK_FP32_NONPACKED_TFLOPS,
        "frac_nonpacked": round(achieved / PEAK_FP32_NONPACKED_TFLOPS, 4) if achieved else None,
        # the tests the kernel executed (its counters), not the model's
        "achieved_executed": round(achieved_exec, 3) if achieved_exec else None,
        "frac_executed": round(achieved_exec / PEAK_FP32_TFLOPS, 4) if achieved_exec else None,
        "frac_executed_nonpacked": round(achieved_exec / PEAK_FP32_NONPACKED_TFLOPS, 4) if achieved_exec else None,
        "kernel_ms": round(kern_ms, 3), "flop_per_sample": round(flop_per_sample, 1),
        "flop_per_sample_executed": round(flop_exec, 1),
        "segments_per_sample": round(s_bar, 4),
        # SURVEY.md 8(d)'s conservative "tests-only" model: S_bar*N*23
        # (linear scenes; the BVH kernel's executed sphere tests otherwise)
        "frac_tests_only": round(tf(23 * model_tests) / PEAK_FP32_TFLOPS, 4) if kern_ms > 0 else None,
        # model: SURVEY.md 8(d)'s N tests per segment (linear); executed: the
        # kernel's own count (for BVH scenes model = executed)
        "model_sphere_tests_per_segment": per_seg(model_tests),
        "sphere_tests_per_segment_executed": per_seg(exec_tests),
        "scan": "linear" if linear else "bvh",
    }
    if linear:
        out["wall_tests_per_segment_executed"] = per_seg(walls)
    else:
        out["box_tests_per_segment"] = per_seg(boxes)
    # measured issue-side view (rocprofv3 profile of this workload,
    # profiles/<tag>_summary.json): wave64 VALU instructions x 2 cycles over
    # the 1,024 SIMDs' cycles -- the hardware bound the FLOP model does not
    # see.  Copied from the committed profile, not measured in this run:
    # profile_head / profile_kernel_hash say which kernel it was taken on,
    # and profile_warning is set when that is not this tree's kernel.
    out.update({
        # FP32 add/mul/fma/trans share of the VALU instructions the profile
        # counted (the rest: compares, selects, moves, integer, converts --
        # real issue slots the FLOP model does not count)
        "valu_fp32_share": pmc.get("valu_fp32_share"),
        "traffic": pmc.get("hbm_bytes_per_launch"),
        "valu_issue_pct_profiled": pmc.get("valu_issue_pct"),
        "profile": pmc.get("tag"),
        "profile_head": pmc.get("commit"),
        "profile_kernel_hash": pmc.get("kernel_hash"),
    })
    here = ptgpu.kernel_source_hash()
    if pmc and pmc.get("kernel_hash") != here:
        out["profile_warning"] = (f"valu_fp32_share / traffic / valu_issue_pct_profiled come from profile "
                                  f"{pmc.get('tag')} (kernel {pmc.get('kernel_hash')}), not this tree's kernel ({here})")
    return s_bar, out


def scan_kernel_name(info):
    """Which render kernel the frame ran (ptg_launch_info)."""
    if info["bvh"]:
        return "bvh"
    return "linear, box mode" if info.get("box_mode") else "linear"


def base_line(args, world, wl_name, scene, W, H, spp, samps, nsub, n_sph, elapsed, parallelism):
    value = W * H * spp * args.steps / elapsed / 1e6
    return value, {
        "metric": metric_of(scene, W, H, spp),
        "value": round(value, 2),
        "unit": "Mray-samples/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f64 (reference-arithmetic mode)" if args.reference_f64 else "f32",
        "data": "synthetic (procedural scene from the reference's box_scene.hpp; counter-RNG seed 0x5EED0001)",
        "config": {"workload": f"{scene} {W}x{H} {spp}spp", "baseline_config": wl_name, "scene": scene,
                   "width": W, "height": H, "spp": spp, "samples_per_subpixel": samps, "num_subpixels": nsub,
                   "spheres": n_sph, "band_rows": args.band_rows, "chunk_samples": args.chunk or "auto",
                   "arithmetic": arith_name(args), "parallelism": parallelism},
    }


def run_inprocess(args):
    """--gpus N > 1 without a launcher (or --launch inprocess): one process,
    ptg_multi over GPUs 0..N-1 (the scene on every device, ONE ncclGather per
    frame over xGMI, the un-shard on GPU 0; csrc/ptg_multi.cpp).  A step is
    one frame kept in HBM.  T1 is the same frame through a one-device
    ptg_multi (render, slab copy -- a device copy, not RCCL -- un-shard),
    timed the same way."""
    n = args.gpus
    rehearsal = os.environ.get("PTG_REHEARSAL") == "1"
    visible = torch.cuda.device_count()
    if not rehearsal and visible < n:
        log(f"error: --gpus {n} needs {n} visible GPUs, {visible} visible (PTG_REHEARSAL=1: {n} shards on GPU 0)")
        sys.exit(2)
    wl_name, scene, W, H, samps, nsub, spp = frame_config(args, n)
    if args.reference_f64:
        log("error: the multi-GPU path renders the fp32 kernel only (--reference-f64 is a 1-GPU parity mode)")
        sys.exit(2)
    scn = ptgpu.make_scene(scene, W, H)
    cam = ptgpu.camera.with_config(scn.camera_parameters)
    n_sph = len(scn.spheres)
    flags = arith_flags(args)
    params = ptgpu.make_params(W, H, samps, nsub, ptgpu.DEFAULT_SEED, args.band_rows, 0, 1, args.chunk, flags=flags)
    cparams = ptgpu.make_params(W, H, samps, nsub, ptgpu.DEFAULT_SEED, args.band_rows, 0, 1, args.chunk,
                                flags=flags | ptgpu.FLAG_COUNT_TESTS)
    mc = ptgpu.MultiContext(scn, cam, list(range(n)), local_shards=n if rehearsal else 0)
    # what the group is: ncclCommCount / ncclCommCuDevice of every communicator
    info = mc.comm_info()
    ranks = [r if r > 0 else None for r, _, _ in info]
    devs = [d for _, d, _ in info]
    bus = [bus_id_of(d) for d in devs]
    bad = check_group(n, ranks if not rehearsal else [], devs, bus, rehearsal)
    if not rehearsal and any(r is None for r in ranks):
        bad.append(f"shards without an RCCL communicator: {info}")
    if bad:
        mc.close()
        log("error: the N-GPU group is not what the line would report: " + "; ".join(bad))
        sys.exit(3)
    counters = mc.frame_device(cparams, counters=True)  # S_bar from the kernels' own counters (untimed)
    seg_total, sph_total, box_total = (int(v) for v in counters[:3])
    for _ in range(max(0, args.warmup - 1)):
        mc.frame_device(params)
    render_ms, frame_ms = [], []
    t0 = time.perf_counter()
    for _ in range(args.steps):
        mc.frame_device(params)  # synchronous: every device done, frame un-sharded on GPU 0
        r, f = mc.frame_timing()
        render_ms.append(r)
        frame_ms.append(f)
    elapsed = time.perf_counter() - t0
    image_n = mc.image(params) if args.t1 == "auto" else None
    mc.close()
    render_ms = np.array(render_ms)  # [steps, n]
    kern_dev = render_ms.mean(0)  # per device

    t1 = None
    if args.t1 == "auto":
        m1 = ptgpu.MultiContext(scn, cam, [0], local_shards=1)
        m1.frame_device(params)  # warm-up
        k1 = max(1, args.t1_steps)
        r1 = []
        w0 = time.perf_counter()
        for _ in range(k1):
            m1.frame_device(params)
            r1.append(m1.frame_timing()[0][0])
        t1_wall = (time.perf_counter() - w0) / k1 * 1e3
        same = bool(np.array_equal(m1.image(params), image_n))
        m1.close()
        t1 = {"wall_ms": round(t1_wall, 3), "kernel_ms": round(float(np.mean(r1)), 3), "frames": k1,
              "image_equals_n_gpu_frame": same}

    frame_samples = W * H * spp
    pmc = load_pmc(f"{scene} {W}x{H} {spp}spp")
    # each device's own share (band rows are not always split evenly): the
    # roofline's `achieved` is the slowest device's samples over its own
    # kernel time
    dev_samples = [int((ptgpu.slab_to_image_rows(H, args.band_rows, k, n) >= 0).sum()) * W * spp for k in range(n)]
    slow = int(np.argmax(kern_dev))
    s_bar, roof = roofline(frame_samples, seg_total, sph_total, box_total, dev_samples[slow], float(kern_dev[slow]),
                           n_sph, pmc)
    par = (f"tile-sharded row bands x{n}, one process (ptg_multi: ncclCommInitAll + ONE ncclGather per frame)"
           + (f" -- REHEARSAL: {n} shards on one GPU, gathered by device copies" if rehearsal else ""))
    value, out = base_line(args, n, wl_name, scene, W, H, spp, samps, nsub, n_sph, elapsed, par)
    out["segments_per_s"] = round(value * 1e6 * s_bar, 1)
    out["roofline"] = roof
    with ptgpu.Context(scn, cam, device=0) as c0:
        out["roofline"]["scan_kernel"] = scan_kernel_name(c0.launch_info(params))
    out["roofline"]["note"] = (f"achieved: the slowest device's kernel (device {devs[slow]}: its {dev_samples[slow]} "
                               f"samples over its HIP-event render time)")
    out["cpu_baseline"] = None
    out["launch"] = "inprocess"
    out["rccl_ranks"] = None if rehearsal else ranks
    out["devices"] = [{"shard": k, "device": d, "pci_bus_id": b, "rccl_user_rank": u}
                      for k, ((_, d, u), b) in enumerate(zip(info, bus))]
    out["group_check"] = ("rehearsal: local shards, no RCCL communicator" if rehearsal else
                          f"ok: {n} RCCL ranks per communicator on {len(set(devs))} distinct devices / "
                          f"{len(set(bus))} PCI bus ids")
    out["per_rank"] = {"render_ms": [round(float(x), 3) for x in kern_dev],
                       "samples": dev_samples,
                       "frame_ms_root": round(float(np.mean(frame_ms)), 3),
                       "note": "HIP events: each device's render; frame_ms_root = GPU 0's render start to the "
                               "end of the gather + un-shard"}
    if t1 is not None:
        tn_wall = elapsed / args.steps * 1e3
        tn_kern = float(render_ms.max(1).mean())  # the slowest shard per frame
        out["t1_ms"] = t1["wall_ms"]
        out["t1"] = dict(t1, note="the same frame on GPU 0 alone through a one-device ptg_multi (its 'gather' is a "
                                  "device copy, the N-GPU step's is RCCL), wall clock per frame like ms_per_step")
        out["efficiency"] = round(t1["wall_ms"] / (n * tn_wall), 4)
        out["efficiency_kernel"] = round(t1["kernel_ms"] / (n * tn_kern), 4)
    print(json.dumps(out), flush=True)


def main(argv=None):
    args = parse_args(argv)
    try:
        mode, world, rank, local = resolve_launch(args.gpus, os.environ)
    except ValueError as e:
        log(f"error: {e}")
        sys.exit(2)
    if mode == "inprocess" or args.launch == "inprocess":
        if world > 1:
            log("error: --launch inprocess drives every GPU from one process; do not start it under a launcher")
            sys.exit(2)
        return run_inprocess(args)
    # PTG_REHEARSAL=1: N ranks on one GPU with gloo (single-GPU box rehearsal
    # of the sharded path); the real multi-GPU run uses nccl (RCCL over xGMI)
    rehearsal = os.environ.get("PTG_REHEARSAL") == "1"
    if rehearsal:
        local = 0
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        if rehearsal:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=dev)

    # what the group is (N > 1): every rank's RCCL communicator (ncclCommCount,
    # device, user rank) and its device's PCI bus id, all-gathered; a group
    # of fewer ranks or distinct devices than --gpus ends the run (exit 3)
    group = None
    if world > 1:
        dist.barrier()  # the communicator exists from here on
        cnt, cdev, urank, why = (None, None, None, "gloo rehearsal: no RCCL communicator") if rehearsal \
            else torch_rccl_info(local)
        bus = bus_id_of(local)
        rec = [cnt if cnt is not None else -1, cdev if cdev is not None else -1, urank if urank is not None else -1,
               local] + list((bus or "").encode()[:32].ljust(32, b"\0"))
        gdev = torch.device("cpu") if rehearsal else dev
        mine = torch.tensor(rec, dtype=torch.int64, device=gdev)
        allr = [torch.zeros_like(mine) for _ in range(world)]
        dist.all_gather(allr, mine)
        recs = [t.cpu().tolist() for t in allr]
        ranks = [r[0] if r[0] >= 0 else None for r in recs]
        buses = [bytes(b for b in r[4:] if b).decode(errors="replace") or None for r in recs]
        # distinct devices: one process per GPU, so the bus ids name them
        bad = check_group(world, ranks, buses, buses, rehearsal)
        group = {"rccl_ranks": None if rehearsal else ranks,
                 "devices": [{"rank": k, "local_rank": r[3], "pci_bus_id": b,
                              "rccl_device": r[1] if r[1] >= 0 else None,
                              "rccl_user_rank": r[2] if r[2] >= 0 else None} for k, (r, b) in enumerate(zip(recs, buses))],
                 "group_check": ("rehearsal: gloo on one GPU, no RCCL communicator" if rehearsal else
                                 ("ok: " if not bad else "FAILED: ") +
                                 f"{world} ranks on {len(set(buses))} distinct PCI bus ids, RCCL ranks {ranks}"
                                 + (f" (ncclCommCount not determinable: {why})" if why and not rehearsal else ""))}
        if bad:
            if rank == 0:
                log("error: the N-GPU group is not what the line would report: " + "; ".join(bad))
            dist.destroy_process_group()
            sys.exit(3)

    wl_name, scene, W, H, samps, nsub, spp = frame_config(args, world)
    scn = ptgpu.make_scene(scene, W, H)
    cam = ptgpu.camera.with_config(scn.camera_parameters)
    ctx = ptgpu.Context(scn, cam, device=local)
    f64 = arith_flags(args)
    params = ptgpu.make_params(W, H, samps, nsub, ptgpu.DEFAULT_SEED, args.band_rows, rank, world, args.chunk,
                               flags=f64)
    cparams = ptgpu.make_params(W, H, samps, nsub, ptgpu.DEFAULT_SEED, args.band_rows, rank, world, args.chunk,
                                flags=ptgpu.FLAG_COUNT_TESTS | f64)
    rows = ptgpu.shard_rows(H, args.band_rows, world)
    slab = torch.zeros(rows * W * 3, dtype=torch.float32, device=dev)
    my_rows = int((ptgpu.slab_to_image_rows(H, args.band_rows, rank, world) >= 0).sum())
    segs = torch.zeros(3, dtype=torch.int64, device=dev)  # scene scans, sphere tests, BVH box tests
    stream = torch.cuda.current_stream(dev)

    def step(count=False, events=None):
        if events is not None:
            events[0].record(stream)
        ctx.render_device(slab, cparams if count else params, segs if count else None, stream)
        if events is not None:
            events[1].record(stream)
        out = slab
        if world > 1:  # the ONE gather (RCCL) + the un-shard on rank 0
            out = ptgpu.render_sharded(params, slab, tile_renderer=lambda out, p: None)
        if events is not None:
            events[2].record(stream)
        return out

    # S_bar from the kernel's own segment counter (untimed)
    step(count=True)
    torch.cuda.synchronize()
    seg_local, sph_local, box_local = (int(v) for v in segs.cpu().tolist())
    if args.reference_f64:  # the reference's linear scan: every sphere per segment (ref64.hpp counts segments only)
        sph_local = seg_local * ctx.n_spheres
    for _ in range(max(0, args.warmup - 1)):
        step()
    torch.cuda.synchronize()

    # N > 1: the same frame rendered by rank 0 alone (shard_count 1), untimed
    # with respect to `value`, timed like a step: wall clock per frame of
    # render + un-shard (the one-slab "gather" is the identity), plus its
    # kernel's HIP events
    t1_frame = None
    if world > 1 and args.t1 == "auto":
        if rank == 0:
            p1 = ptgpu.make_params(W, H, samps, nsub, ptgpu.DEFAULT_SEED, args.band_rows, 0, 1, args.chunk, flags=f64)
            full = torch.empty(ptgpu.shard_rows(H, args.band_rows, 1) * W * 3, dtype=torch.float32, device=dev)
            img1 = torch.empty((H, W, 3), dtype=torch.float32, device=dev)
            ctx.render_device(full, p1, None, stream)  # warm-up (allocates the accumulator)
            torch.cuda.synchronize()
            k1 = max(1, args.t1_steps)
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(k1)]
            w0 = time.perf_counter()
            for e0, e1 in ev:
                e0.record(stream)
                ctx.render_device(full, p1, None, stream)
                e1.record(stream)
                ptgpu.unshard_device(full, img1, W, H, args.band_rows, 1, stream)
                torch.cuda.synchronize()
            t1_frame = {"wall_ms": round((time.perf_counter() - w0) / k1 * 1e3, 3),
                        "kernel_ms": round(float(np.mean([a.elapsed_time(b) for a, b in ev])), 3), "frames": k1}
            del full, img1
        dist.barrier()

    evs = [tuple(torch.cuda.Event(enable_timing=True) for _ in range(3)) for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(events=evs[i])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    kern_ms = float(np.mean([a.elapsed_time(b) for a, b, _ in evs])) if args.steps else float("nan")
    gather_ms = float(np.mean([b.elapsed_time(c) for _, b, c in evs])) if args.steps else float("nan")
    per_rank = None
    kern_max = kern_ms
    if world > 1:  # per-rank render and gather (+ un-shard on rank 0) times, HIP events on the launch stream
        cdev0 = torch.device("cpu") if rehearsal else dev
        mine = torch.tensor([kern_ms, gather_ms], dtype=torch.float64, device=cdev0)
        allr = [torch.zeros_like(mine) for _ in range(world)]
        dist.all_gather(allr, mine)
        per_rank = {"render_ms": [round(float(t[0]), 3) for t in allr],
                    "gather_ms": [round(float(t[1]), 3) for t in allr],
                    "note": "gather_ms: the RCCL gather (and rank 0's un-shard), incl. waiting for the slowest rank"}
        kern_max = max(float(t[0]) for t in allr)

    seg_total = seg_local
    if world > 1:
        cdev = torch.device("cpu") if rehearsal else dev
        t = torch.tensor([elapsed], dtype=torch.float64, device=cdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t[0])
        s = torch.tensor([seg_local, sph_local, box_local], dtype=torch.int64, device=cdev)
        dist.all_reduce(s)
        seg_total, sph_local, box_local = (int(v) for v in s.cpu().tolist())

    if rank == 0:
        frame_samples = W * H * spp
        pmc = load_pmc(f"{scene} {W}x{H} {spp}spp")
        s_bar, roof = roofline(frame_samples, seg_total, sph_local, box_local, my_rows * W * spp, kern_ms,
                               ctx.n_spheres, pmc)
        par = ((f"tile-sharded row bands x{world}, one process per GPU (torch.distributed nccl = RCCL)"
                + (" (gloo rehearsal on one GPU)" if rehearsal else "")) if world > 1 else "single GPU")
        value, out = base_line(args, world, wl_name, scene, W, H, spp, samps, nsub, ctx.n_spheres, elapsed, par)
        out["segments_per_s"] = round(value * 1e6 * s_bar, 1)
        out["roofline"] = roof
        out["roofline"]["scan_kernel"] = scan_kernel_name(ctx.launch_info(params))
        cpu = None
        if world == 1 and args.cpu_baseline == "auto":
            frame = slab.cpu().numpy().reshape(rows, W, 3)[:H]  # band_rows = 1, one shard: slab row = image row
            cpu = cpu_baseline(scene, W, H, samps, nsub, args.cpu_threads or default_cpu_threads(),
                               max(1, args.cpu_row_step), frame, ptgpu.DEFAULT_SEED, args.quality_rows)
        out["cpu_baseline"] = cpu
        out["launch"] = "torchrun" if world > 1 else "single"
        if group is not None:
            out.update(group)
        if per_rank is not None:
            out["per_rank"] = per_rank
        if t1_frame is not None:
            tn_wall = elapsed / args.steps * 1e3
            out["t1_ms"] = t1_frame["wall_ms"]
            out["t1"] = dict(t1_frame, note="the same frame on rank 0's GPU alone (render + un-shard), wall clock "
                                            "per frame like ms_per_step; kernel_ms from HIP events")
            out["efficiency"] = round(t1_frame["wall_ms"] / (world * tn_wall), 4)
            out["efficiency_kernel"] = round(t1_frame["kernel_ms"] / (world * kern_max), 4)
        if cpu:
            out["speedup_vs_cpu_baseline"] = round(value / cpu["value"], 1)
        print(json.dumps(out), flush=True)
    ctx.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
