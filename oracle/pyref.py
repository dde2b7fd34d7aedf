"""pyref.py -- TEST INFRASTRUCTURE ONLY.

ctypes binding of oracle/_ref/libref_main.so: the REFERENCE's own
src/main.cpp:27-197 (intersect, diffuse/specular/dielectric_ray, radiance,
render_subpixel) compiled with its `pt` library by oracle/Makefile (see
oracle/ref_main_capi.cpp).  Used by oracle/gen_ref_paths.py (golden fixtures),
by tests that pin the oracle directly when the library is present, and by
bench.py's cpu_baseline leg (kind "reference": the reference's own per-pixel
code in an OpenMP row loop).  The product path never imports this module.

_ref/ is built in this container (it needs /root/reference) and travels to
the GPU box with the tree like every built .so; `available()` is False where
it was not built.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_ref", "libref_main.so")

_lib = None


def available() -> bool:
    return os.path.exists(LIB_PATH)


def lib():
    global _lib
    if _lib is None:
        if not available():
            raise FileNotFoundError(f"{LIB_PATH} missing: run `make -C oracle ref` where /root/reference exists")
        L = C.CDLL(LIB_PATH)
        P, D, I, U32 = C.c_void_p, C.c_double, C.c_int, C.c_uint32
        sig = {
            "ref_abi_version": (I, []),
            "ref_intersect_scene": (I, [P, I, P, P, P, P]),
            "ref_brdf": (I, [I, P, P, P, D, U32, P, P, P]),
            "ref_paths": (I, [P, I, P, U32, I, I, P, P, P, P]),
            "ref_render_rows": (I, [P, I, P, I, I, I, I, P, I, I, I, I, P]),
        }
        for name, (res, args) in sig.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        assert L.ref_abi_version() == 1
        _lib = L
    return _lib


def _p(a: np.ndarray):
    assert a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(C.c_void_p)


def _v(x) -> np.ndarray:
    return np.ascontiguousarray(np.asarray(x, dtype=np.float64).reshape(3))


def intersect_scene(spheres, o, d):
    """main.cpp:30-42: (hit, t, id)."""
    t = np.zeros(1)
    i = np.zeros(1, dtype=np.int64)
    hit = lib().ref_intersect_scene(_p(spheres), len(spheres), _p(_v(o)), _p(_v(d)), _p(t), _p(i))
    return bool(hit), float(t[0]), int(i[0])


BRDF_KINDS = {"diffuse": 0, "specular": 1, "dielectric": 2}


def brdf(kind: str, sphere, o, d, t: float, seed: int):
    """diffuse_ray / specular_ray / dielectric_ray (main.cpp:44-97) on
    get_hit_record_at(sphere, ray(o, d), t): (origin, direction, draws, next)."""
    one = np.ascontiguousarray(np.asarray(sphere).reshape(1))
    ro, rd, nxt = np.zeros(3), np.zeros(3), np.zeros(1)
    draws = lib().ref_brdf(BRDF_KINDS[kind], _p(one), _p(_v(o)), _p(_v(d)), float(t), seed & 0xFFFFFFFF,
                           _p(ro), _p(rd), _p(nxt))
    assert draws >= 0
    return ro, rd, draws, float(nxt[0])


def paths(spheres, cam, seed0: int, count: int, nthreads: int = 8):
    """count camera paths, path k on mt19937(seed0 + k): s, t = 2 draws,
    get_ray, radiance.  Returns (rays [count, 6], values [count, 3],
    draws [count], next [count])."""
    rays = np.zeros((count, 6))
    vals = np.zeros((count, 3))
    draws = np.zeros(count, dtype=np.int32)
    nxt = np.zeros(count)
    assert lib().ref_paths(_p(spheres), len(spheres), _p(cam), seed0 & 0xFFFFFFFF, count, nthreads, _p(rays),
                           _p(vals), _p(draws), _p(nxt)) == 0
    return rays, vals, draws, nxt


def reference_row_seeds(H: int, rd_value: int) -> np.ndarray:
    """main.cpp:222-223 + random_state.cpp:5: mt19937(random_device()() *
    (unsigned short)(y*y*y)), with rd_value standing in for random_device()()."""
    y = np.arange(H, dtype=np.uint64)
    return ((((y * y * y) & 0xFFFF) * np.uint64(rd_value & 0xFFFFFFFF)) & 0xFFFFFFFF).astype(np.uint32)


def render_rows(spheres, cam, W, H, samps, nsub, row_seeds, rows=None, nthreads=8, image=None):
    """The reference row loop (main.cpp:217-234 task body, OpenMP over rows):
    image [H, W, 3] doubles in the reference's row order, added into."""
    y0, y1, ys = rows if rows is not None else (0, H, 1)
    seeds = np.ascontiguousarray(row_seeds, dtype=np.uint32)
    assert seeds.size == H
    img = np.zeros(W * H * 3) if image is None else np.ascontiguousarray(image, dtype=np.float64).reshape(-1)
    assert lib().ref_render_rows(_p(spheres), len(spheres), _p(cam), W, H, samps, nsub, _p(seeds), y0, y1, ys,
                                 nthreads, _p(img)) == 0
    return img.reshape(H, W, 3)
