"""Host-side render API over the C ABI.

* render(...)            -- the drop-in for the reference's row loop
                            (main.cpp:214-236): fills the caller's image
                            (H*W RGB doubles, reference row order) exactly as
                            the loop would, through ptg_render.
* Context                -- device-resident scene for repeated renders into
                            torch CUDA tensors (bench, multi-GPU).
* render_sharded(...)    -- one process per GPU: each rank renders its
                            interleaved row bands into a slab, one gather
                            (RCCL over xGMI via torch.distributed) collects
                            the slabs on rank 0, ptg_unshard_device restores
                            the row order.
"""
from __future__ import annotations

import ctypes as C
from typing import Callable, Optional

import numpy as np

from ._abi import Params, check, lib
from .scene import CAMERA_DT, SPHERE_DT, camera, scene

DEFAULT_SEED = 0x5EED0001
DEFAULT_BAND_ROWS = 1  # single-row bands: equal shards whenever N divides H (tools/shard_sim.py: 8-way 95.8 % vs 94.4 % with 8-row bands)


def _spheres_array(scn) -> np.ndarray:
    if isinstance(scn, scene):
        return scn.to_array()
    a = np.ascontiguousarray(scn)
    if a.dtype != SPHERE_DT:
        raise TypeError("spheres must be a ptgpu.scene or a SPHERE_DT array")
    return a


def _camera_array(cam) -> np.ndarray:
    if isinstance(cam, camera):
        return cam.to_array()
    a = np.ascontiguousarray(cam).reshape(1)
    if a.dtype != CAMERA_DT:
        raise TypeError("cam must be a ptgpu.camera or a CAMERA_DT array")
    return a


FLAG_COUNT_TESTS = 1  # include/ptgpu.h PTG_FLAG_COUNT_TESTS
FLAG_COUNT_NONFINITE = 2  # include/ptgpu.h PTG_FLAG_COUNT_NONFINITE (4 counters)
FLAG_REFERENCE_F64 = 4  # include/ptgpu.h PTG_FLAG_REFERENCE_F64: the reference's double arithmetic (parity mode)
FLAG_EXACT_MATH = 8  # include/ptgpu.h PTG_FLAG_EXACT_MATH: exact sequences, bit for bit the oracle's Mode B


def _n_counters(flags: int) -> int:
    return 4 if flags & FLAG_COUNT_NONFINITE else (3 if flags & FLAG_COUNT_TESTS else 1)


def make_params(width, height, samples, num_subpixels=2, seed=DEFAULT_SEED, band_rows=DEFAULT_BAND_ROWS,
                shard_rank=0, shard_count=1, chunk_samples=0, flags=0) -> Params:
    return Params(int(width), int(height), int(samples), int(num_subpixels), int(seed) & (2**64 - 1),
                  int(band_rows), int(shard_rank), int(shard_count), int(chunk_samples), int(flags))


def shard_rows(height: int, band_rows: int, shard_count: int) -> int:
    out = C.c_int32(0)
    check(lib().ptg_shard_rows(height, band_rows, shard_count, C.byref(out)), "ptg_shard_rows")
    return out.value


def slab_to_image_rows(height: int, band_rows: int, shard_rank: int, shard_count: int) -> np.ndarray:
    """Output row of every slab row (-1 for padding), the mapping ptg_render_device uses."""
    rows = shard_rows(height, band_rows, shard_count)
    j = np.arange(rows)
    band = j // band_rows
    r = (band * shard_count + shard_rank) * band_rows + (j - band * band_rows)
    return np.where(r < height, r, -1)


def unshard_host(gathered: np.ndarray, width: int, height: int, band_rows: int, shard_count: int) -> np.ndarray:
    """Host statement of ptg_unshard_device (rank-major slabs -> image rows)."""
    rows = shard_rows(height, band_rows, shard_count)
    g = np.asarray(gathered).reshape(shard_count * rows, width * 3)
    out = np.zeros((height, width * 3), dtype=g.dtype)
    for k in range(shard_count):
        m = slab_to_image_rows(height, band_rows, k, shard_count)
        ok = m >= 0
        out[m[ok]] = g[k * rows:(k + 1) * rows][ok]
    return out.reshape(height, width, 3)


def render(scn, cam, image: np.ndarray, width: int, height: int, samples: int, num_subpixels: int = 2,
           seed: int = DEFAULT_SEED, device: int = -1, flags: int = 0) -> np.ndarray:
    """Drop-in for main.cpp:214-236: image (W*H RGB doubles, reference row
    order, zero-initialised by the caller like main.cpp:210-212) receives
    += sum_sub clamp(mean radiance) / num_subpixels^2 for every pixel."""
    sp = _spheres_array(scn)
    ca = _camera_array(cam)
    img = image if image.dtype == np.float64 and image.flags["C_CONTIGUOUS"] else None
    if img is None or img.size != width * height * 3:
        raise ValueError("image must be a C-contiguous float64 array of width*height*3 values")
    p = make_params(width, height, samples, num_subpixels, seed, flags=flags)
    check(lib().ptg_render(sp.ctypes.data_as(C.c_void_p), len(sp), ca.ctypes.data_as(C.c_void_p), C.byref(p),
                           int(device), img.ctypes.data_as(C.c_void_p)), "ptg_render")
    return image


def render_multi(scn, cam, image: np.ndarray, width: int, height: int, samples: int, devices,
                 num_subpixels: int = 2, seed: int = DEFAULT_SEED, band_rows: int = DEFAULT_BAND_ROWS,
                 flags: int = 0) -> np.ndarray:
    """ptg_render_multi: the drop-in render over several GPUs of this process
    (distinct devices) -- shards rendered concurrently, ONE RCCL gather to
    devices[0], un-shard there; the image equals render()'s bit for bit."""
    sp = _spheres_array(scn)
    ca = _camera_array(cam)
    if image.dtype != np.float64 or not image.flags["C_CONTIGUOUS"] or image.size != width * height * 3:
        raise ValueError("image must be a C-contiguous float64 array of width*height*3 values")
    p = make_params(width, height, samples, num_subpixels, seed, band_rows, flags=flags)
    devs = (C.c_int * len(devices))(*[int(d) for d in devices])
    check(lib().ptg_render_multi(sp.ctypes.data_as(C.c_void_p), len(sp), ca.ctypes.data_as(C.c_void_p), C.byref(p),
                                 devs, len(devices), image.ctypes.data_as(C.c_void_p)), "ptg_render_multi")
    return image


class MultiContext:
    """A persistent multi-GPU context (ptg_multi): the scene on every device,
    the RCCL communicator of the device set, the root's gather buffers --
    repeated frames and progressive passes reuse them.  `local_shards=n`
    (tests) puts n shards on the one device `devices[0]`, gathered by device
    copies into the layout an n-rank ncclGather produces."""

    def __init__(self, scn, cam, devices, local_shards: int = 0):
        sp = _spheres_array(scn)
        ca = _camera_array(cam)
        h = C.c_void_p()
        if local_shards:
            check(lib().ptg_multi_create_local_(sp.ctypes.data_as(C.c_void_p), len(sp), ca.ctypes.data_as(C.c_void_p),
                                                int(devices[0]), int(local_shards), C.byref(h)),
                  "ptg_multi_create_local_")
        else:
            devs = (C.c_int * len(devices))(*[int(d) for d in devices])
            check(lib().ptg_multi_create(sp.ctypes.data_as(C.c_void_p), len(sp), ca.ctypes.data_as(C.c_void_p), devs,
                                         len(devices), C.byref(h)), "ptg_multi_create")
        self._h = h
        self.n_devices = int(local_shards) if local_shards else len(devices)

    def close(self):
        if self._h:
            lib().ptg_multi_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    @staticmethod
    def _image(image, params, dtype):
        if image.dtype != dtype or not image.flags["C_CONTIGUOUS"] or \
                image.size != params.width * params.height * 3:
            raise ValueError(f"image must be a C-contiguous {np.dtype(dtype).name} array of width*height*3 values")
        return image.ctypes.data_as(C.c_void_p)

    def render(self, image: np.ndarray, params: Params) -> np.ndarray:
        """The frame over all devices, added into `image` (float64, like render())."""
        check(lib().ptg_multi_render(self._h, C.byref(params), self._image(image, params, np.float64)),
              "ptg_multi_render")
        return image

    def frame_device(self, params: Params, counters: bool = False):
        """ptg_multi_frame_device: the frame over all devices, kept in HBM
        (render, ONE gather, un-shard; synchronous).  With counters=True
        (params needs FLAG_COUNT_TESTS) returns the 4 summed kernel counters."""
        c = np.zeros(4, dtype=np.uint64)
        check(lib().ptg_multi_frame_device(self._h, C.byref(params), c.ctypes.data_as(C.c_void_p) if counters else None),
              "ptg_multi_frame_device")
        return c if counters else None

    def frame_timing(self):
        """(render_ms per device, frame_ms on the root) of the last frame_device."""
        r = np.zeros(self.n_devices, dtype=np.float32)
        f = np.zeros(1, dtype=np.float32)
        check(lib().ptg_multi_frame_timing(self._h, r.ctypes.data_as(C.c_void_p), self.n_devices,
                                           f.ctypes.data_as(C.c_void_p)), "ptg_multi_frame_timing")
        return r.astype(float).tolist(), float(f[0])

    def image(self, params: Params) -> np.ndarray:
        """The last frame_device image, [H, W, 3] float32 in the reference's row order."""
        out = np.empty(params.width * params.height * 3, dtype=np.float32)
        check(lib().ptg_multi_image(self._h, C.byref(params), out.ctypes.data_as(C.c_void_p)), "ptg_multi_image")
        return out.reshape(params.height, params.width, 3)

    def comm_info(self):
        """ptg_multi_comm_info: per shard (ncclCommCount, ncclCommCuDevice,
        ncclCommUserRank) of its RCCL communicator -- (0, the shard's device,
        -1) for local shards (no communicator)."""
        n = self.n_devices
        ranks = np.zeros(n, dtype=np.int32)
        devs = np.zeros(n, dtype=np.int32)
        user = np.zeros(n, dtype=np.int32)
        check(lib().ptg_multi_comm_info(self._h, ranks.ctypes.data_as(C.c_void_p), devs.ctypes.data_as(C.c_void_p),
                                        user.ctypes.data_as(C.c_void_p), n), "ptg_multi_comm_info")
        return [(int(r), int(d), int(u)) for r, d, u in zip(ranks, devs, user)]

    def inject_gather_fault_(self, shard: int) -> None:
        """Tests: the next RCCL gather fails at `shard` (-1: off)."""
        check(lib().ptg_multi_inject_gather_fault_(self._h, int(shard)), "ptg_multi_inject_gather_fault_")

    def reset_accumulation(self, params: Params) -> None:
        check(lib().ptg_multi_reset_accumulation(self._h, C.byref(params)), "ptg_multi_reset_accumulation")

    def accumulate(self, params: Params, sample_begin: int, sample_end: int) -> None:
        check(lib().ptg_multi_accumulate(self._h, C.byref(params), int(sample_begin), int(sample_end)),
              "ptg_multi_accumulate")

    def resolve(self, image: np.ndarray, params: Params, samples_done: int) -> np.ndarray:
        """The image of the samples accumulated so far, written to `image` (float32)."""
        check(lib().ptg_multi_resolve(self._h, C.byref(params), int(samples_done),
                                      self._image(image, params, np.float32)), "ptg_multi_resolve")
        return image


KERNEL_SOURCES = ("ptg_render.hip", "pt_device.hpp", "bvh_build.hpp")


def kernel_source_hash() -> str:
    """sha256 (12 hex digits) of the render kernels' sources (csrc/): names
    the kernel a committed rocprofv3 profile was taken on (profiles/
    summarize.py records it, bench.py compares it with this tree's)."""
    import hashlib
    import os
    h = hashlib.sha256()
    src = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "csrc")
    for name in KERNEL_SOURCES:
        try:
            with open(os.path.join(src, name), "rb") as f:
                h.update(f.read())
        except OSError:
            return "unavailable"
    return h.hexdigest()[:12]


def pci_bus_id(device: int) -> str:
    """ptg_device_pci_bus_id: the PCI bus id of HIP device `device`."""
    buf = C.create_string_buffer(64)
    check(lib().ptg_device_pci_bus_id(int(device), buf, len(buf)), "ptg_device_pci_bus_id")
    return buf.value.decode()


def scene_layout(scn, cam):
    """Host-side scene preparation (ptg_scene_layout, no device needed): the
    anchor axis of each huge sphere (-1: camera-facing anchor, or not huge)
    and the linear scan order (scene indices in the order they are tested)."""
    sp = _spheres_array(scn)
    ca = _camera_array(cam)
    n = len(sp)
    axis = np.zeros(max(n, 1), dtype=np.int32)
    order = np.zeros(max(n, 1), dtype=np.int32)
    check(lib().ptg_scene_layout(sp.ctypes.data, n, ca.ctypes.data, axis.ctypes.data, order.ctypes.data),
          "ptg_scene_layout")
    return axis[:n].tolist(), order[:n].tolist()


class Context:
    """A scene prepared in HBM on one device (ptg_context)."""

    def __init__(self, scn, cam, device: Optional[int] = None):
        sp = _spheres_array(scn)
        ca = _camera_array(cam)
        h = C.c_void_p()
        check(lib().ptg_context_create(sp.ctypes.data_as(C.c_void_p), len(sp), ca.ctypes.data_as(C.c_void_p),
                                       -1 if device is None else int(device), C.byref(h)), "ptg_context_create")
        self._h = h
        self.n_spheres = len(sp)
        if device is None or int(device) < 0:
            import torch
            device = torch.cuda.current_device() if torch.cuda.is_available() else 0
        self.device = int(device)

    def _stream(self, stream):
        """The HIP stream handle: `stream`, or torch's current stream on the
        context's device (not the current device)."""
        import torch
        return (stream or torch.cuda.current_stream(torch.device("cuda", self.device))).cuda_stream

    def _check(self, t, dtype, min_numel):
        _check_tensor(t, dtype, min_numel)
        if t.device.index != self.device:
            raise ValueError(f"tensor on {t.device}, context on cuda:{self.device}")

    def close(self):
        if self._h:
            lib().ptg_context_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def render_device(self, out, params: Params, segments=None, stream=None) -> None:
        """Asynchronous render into `out` (torch float32 CUDA tensor of
        shard_rows*W*3 values) on `stream` (torch.cuda.Stream or None =
        torch's current stream)."""
        import torch
        self._check(out, torch.float32, shard_rows(params.height, params.band_rows, params.shard_count)
                    * params.width * 3)
        if segments is not None:
            self._check(segments, torch.int64, _n_counters(params.flags))
        s = self._stream(stream)
        check(lib().ptg_render_device(self._h, C.byref(params), C.c_void_p(out.data_ptr()),
                                      C.c_void_p(segments.data_ptr()) if segments is not None else None,
                                      C.c_void_p(s)), "ptg_render_device")

    LAUNCH_INFO = ("box_mode", "box_walls_out", "bvh", "units", "workgroups", "levels", "resolve_pass",
                   "wall_pairs")  # include/ptgpu.h ptg_launch_info

    def launch_info(self, params: Params) -> dict:
        """ptg_launch_info: how ptg_render_device would launch this frame
        (scan mode, work units, levels) -- host-side, nothing is launched."""
        v = np.zeros(len(self.LAUNCH_INFO), dtype=np.int64)
        check(lib().ptg_launch_info(self._h, C.byref(params), v.ctypes.data_as(C.c_void_p), len(v)),
              "ptg_launch_info")
        return dict(zip(self.LAUNCH_INFO, (int(x) for x in v)))

    # ---- progressive accumulation (ptg_accumulate_device / ptg_resolve_device)
    def reset_accumulation(self, params: Params, stream=None) -> None:
        s = self._stream(stream)
        check(lib().ptg_reset_accumulation_device(self._h, C.byref(params), C.c_void_p(s)), "ptg_reset_accumulation_device")

    def accumulate(self, params: Params, sample_begin: int, sample_end: int, segments=None, stream=None) -> None:
        """Add samples [sample_begin, sample_end) of every sub-pixel."""
        import torch
        if segments is not None:
            self._check(segments, torch.int64, _n_counters(params.flags))
        s = self._stream(stream)
        check(lib().ptg_accumulate_device(self._h, C.byref(params), int(sample_begin), int(sample_end),
                                          C.c_void_p(segments.data_ptr()) if segments is not None else None,
                                          C.c_void_p(s)), "ptg_accumulate_device")

    def resolve(self, out, params: Params, samples_done: int, stream=None) -> None:
        """Preview/final image from the samples accumulated so far."""
        import torch
        self._check(out, torch.float32, shard_rows(params.height, params.band_rows, params.shard_count)
                    * params.width * 3)
        s = self._stream(stream)
        check(lib().ptg_resolve_device(self._h, C.byref(params), int(samples_done), C.c_void_p(out.data_ptr()),
                                       C.c_void_p(s)), "ptg_resolve_device")

    def trace_samples(self, coords, params: Params):
        """Parity probe: radiance + segment count of individual paths
        (coords: int32 CUDA tensor [n, 5] = x, y, sx, sy, sample)."""
        import torch
        if coords.dim() != 2 or coords.shape[1] != 5:
            raise ValueError("coords must be [n, 5] (x, y, sx, sy, sample)")
        coords = coords.contiguous()
        self._check(coords, torch.int32, coords.numel())
        n = coords.shape[0]
        out = torch.empty((n, 3), dtype=torch.float32, device=coords.device)
        segs = torch.empty((n,), dtype=torch.int32, device=coords.device)
        s = self._stream(None)
        check(lib().ptg_trace_samples_device(self._h, C.byref(params), C.c_void_p(coords.data_ptr()), n,
                                             C.c_void_p(out.data_ptr()), C.c_void_p(segs.data_ptr()),
                                             C.c_void_p(s)), "ptg_trace_samples_device")
        return out, segs

    PROBE_OPS = {"sqrt": 0, "rsqrt": 1, "div": 2, "sincos": 3}  # include/ptgpu.h PTG_PROBE_*

    def math_probe(self, op: str, x, exact: bool):
        """The kernels' arithmetic primitive `op` on a float32 CUDA tensor:
        sqrt / rsqrt of x [n]; div of x [n, 2] (x[:, 0] / x[:, 1]); sincos of
        24-bit integers m (x: int32 [n]) -> [n, 2] (cos, sin of 2 pi m 2^-24)."""
        import torch
        code = self.PROBE_OPS[op]
        x = x.contiguous()
        if op == "div":
            if x.dim() != 2 or x.shape[1] != 2:
                raise ValueError("div takes [n, 2] operands")
            n = x.shape[0]
        else:
            n = x.numel()
        if op == "sincos":
            self._check(x, torch.int32, n)
            x = x.view(torch.float32)
        else:
            self._check(x, torch.float32, x.numel())
        out = torch.empty((n, 2) if op == "sincos" else (n,), dtype=torch.float32, device=x.device)
        s = self._stream(None)
        check(lib().ptg_math_probe_device(self._h, code, 1 if exact else 0, C.c_void_p(x.data_ptr()),
                                          C.c_void_p(out.data_ptr()), n, C.c_void_p(s)), "ptg_math_probe_device")
        return out


def _check_tensor(t, dtype, min_numel):
    if not t.is_cuda or t.dtype != dtype or not t.is_contiguous() or t.numel() < min_numel:
        raise ValueError(f"expected a contiguous CUDA {dtype} tensor with >= {min_numel} elements")


def unshard_device(gathered, image, width, height, band_rows, shard_count, stream=None):
    import torch
    s = (stream or torch.cuda.current_stream(image.device)).cuda_stream
    check(lib().ptg_unshard_device(C.c_void_p(gathered.data_ptr()), C.c_void_p(image.data_ptr()), width, height,
                                   band_rows, shard_count, C.c_void_p(s)), "ptg_unshard_device")


def tonemap_device(image, out_u8, stream=None):
    """utils.cpp:11-16 on the GPU: uint8 gamma-2.2 values of every channel."""
    import torch
    s = (stream or torch.cuda.current_stream(image.device)).cuda_stream
    check(lib().ptg_tonemap_device(C.c_void_p(image.data_ptr()), C.c_void_p(out_u8.data_ptr()), image.numel(),
                                   C.c_void_p(s)), "ptg_tonemap_device")


def render_sharded(params: Params, slab, group=None,
                   tile_renderer: Optional[Callable] = None, ctx: Optional[Context] = None,
                   unshard: Optional[Callable] = None):
    """One rank's part of a tile-sharded frame.

    Renders this rank's bands into `slab`, then ONE gather collects every
    slab on rank 0 (torch.distributed: RCCL over xGMI on the nccl backend,
    gloo on CPU).  Rank 0 returns the reassembled image tensor [H, W, 3];
    other ranks return None.  `tile_renderer(slab, params)` defaults to the
    HIP megakernel (ctx.render_device); tests substitute a CPU renderer to
    exercise the sharding logic with gloo."""
    import torch
    import torch.distributed as dist
    if tile_renderer is None:
        if ctx is None:
            raise ValueError("render_sharded needs ctx (HIP path) or tile_renderer")
        tile_renderer = lambda out, p: ctx.render_device(out, p)  # noqa: E731
    tile_renderer(slab, params)
    rank = dist.get_rank(group)
    world = dist.get_world_size(group)
    assert params.shard_count == world and params.shard_rank == rank
    # gloo cannot gather device tensors: stage through host memory (CPU
    # rehearsals only; the nccl backend (RCCL) gathers HBM to HBM over xGMI)
    staged = slab.is_cuda and dist.get_backend(group) == "gloo"
    send = slab.cpu() if staged else slab
    if rank == 0:
        gathered = torch.empty((world,) + tuple(send.shape), dtype=send.dtype, device=send.device)
        dist.gather(send, gather_list=list(gathered.unbind(0)), dst=0, group=group)
        if staged:
            gathered = gathered.to(slab.device)
        image = torch.empty((params.height, params.width, 3), dtype=slab.dtype, device=slab.device)
        if unshard is not None:
            unshard(gathered, image, params)
        elif slab.is_cuda:
            unshard_device(gathered, image, params.width, params.height, params.band_rows, world)
        else:
            image.copy_(torch.from_numpy(unshard_host(gathered.numpy(), params.width, params.height,
                                                       params.band_rows, world)))
        return image
    dist.gather(send, gather_list=None, dst=0, group=group)
    return None
