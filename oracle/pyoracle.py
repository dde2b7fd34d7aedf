"""pyoracle.py -- TEST INFRASTRUCTURE ONLY.

ctypes binding of oracle/libpt_oracle.so (the C restatement of the
reference's hot path, see pt_oracle.h).  Imported only by tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg -- the product path
(cpu-path-tracing_amd/ptgpu) never imports this module.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libpt_oracle.so")

# numpy mirrors of po_sphere / po_camera_config / po_camera (= pt::sphere,
# pt::camera_config, pt::camera layouts: sphere.hpp:10-17, camera.hpp:11-33)
SPHERE_DT = np.dtype([("radius", "<f8"), ("position", "<f8", 3), ("emission", "<f8", 3),
                      ("color", "<f8", 3), ("material", "<i4"), ("pad_", "<i4")])
CAMCFG_DT = np.dtype([("position", "<f8", 3), ("direction", "<f8", 3), ("up", "<f8", 3),
                      ("aspect_ratio", "<f8"), ("vertical_fov_radians", "<f8"),
                      ("focal_length", "<f8"), ("aperture", "<f8"), ("focus_distance", "<f8")])
CAMERA_DT = np.dtype([("position", "<f8", 3), ("lower_left_corner", "<f8", 3),
                      ("cam_x_axis", "<f8", 3), ("cam_y_axis", "<f8", 3), ("u", "<f8", 3),
                      ("v", "<f8", 3), ("w", "<f8", 3), ("lens_radius", "<f8")])
assert SPHERE_DT.itemsize == 88 and CAMCFG_DT.itemsize == 112 and CAMERA_DT.itemsize == 176

MT_STATE_BYTES = 624 * 4 + 4

SCENES = {"simple": 0, "box": 1, "box_mirror": 2}

_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise FileNotFoundError(f"{LIB_PATH} missing: run `make -C oracle`")
        L = C.CDLL(LIB_PATH)
        P = C.c_void_p
        D = C.c_double
        I = C.c_int
        U32 = C.c_uint32
        U64 = C.c_uint64
        sig = {
            "po_mt_seed": (None, [P, U32]),
            "po_mt_next": (U32, [P]),
            "po_mt_generate": (D, [P]),
            "po_mt_generate_between": (D, [P, D, D]),
            "po_camera_with_config": (None, [P, P]),
            "po_camera_get_ray_mt": (I, [P, D, D, P, P, P]),
            "po_sphere_intersect": (D, [P, P, P]),
            "po_hit_record": (None, [P, P, P, D, P]),
            "po_clamp": (D, [D]),
            "po_color_to_int": (I, [D]),
            "po_vec_length": (D, [P]),
            "po_scene": (I, [I, I, I, P, I, P]),
            "po_scene_synthetic": (I, [I, I, I, U32, P, P]),
            "po_intersect_scene": (I, [P, I, P, P, P, P]),
            "po_diffuse_ray_mt": (I, [P, P, P, P, P, P]),
            "po_specular_ray_mt": (I, [P, P, P, P, P, P]),
            "po_dielectric_ray_mt": (I, [P, P, P, P, P, P]),
            "po_radiance_mt": (I, [P, I, P, P, P, P]),
            "po_render_mt": (I, [P, I, P, I, I, I, I, U32, I, I, I, I, P]),
            "po_key_hash": (U64, [U64, U64]),
            "po_sample_state": (U32, [U64, U32]),
            "po_xorshift32": (U32, [P]),
            "po_render_xs_f64": (I, [P, I, P, I, I, I, I, U64, I, I, I, I, P, P]),
            "po_render_xs_f32": (I, [P, I, P, I, I, I, I, U64, I, I, I, I, P, P]),
            "po_render_xs_f32_ex": (I, [P, I, P, I, I, I, I, U64, I, I, I, I, P, P, P]),
            "po_render_xs_f64_rect": (I, [P, I, P, I, I, I, I, U64, I, I, I, I, I, I, P, P]),
            "po_render_xs_f32_rect": (I, [P, I, P, I, I, I, I, U64, I, I, I, I, I, I, P, P]),
            "po_sample_f32": (I, [P, I, P, I, I, I, U64, I, I, I, I, U32, P]),
            "po_tonemap": (None, [P, C.c_size_t, P]),
            "po_scan_layout": (I, [P, I, P, P, P]),
            "po_sincos2pi": (None, [P, C.c_size_t, P]),
            "po_mode_b_math": (None, [P, P, C.c_size_t, P, P]),
            "po_mode_b_roots": (None, [P, C.c_size_t, P, P]),
            "po_set_mode_b_variant": (None, [I]),
            "po_get_mode_b_variant": (I, []),
        }
        for name, (res, args) in sig.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def ptr(a: np.ndarray):
    assert a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(C.c_void_p)


def vec(x) -> np.ndarray:
    return np.ascontiguousarray(np.asarray(x, dtype=np.float64).reshape(3))


# ---------------------------------------------------------------- L0 / rng
class MT19937:
    def __init__(self, seed: int):
        self.buf = np.zeros(MT_STATE_BYTES, dtype=np.uint8)
        lib().po_mt_seed(ptr(self.buf), seed & 0xFFFFFFFF)

    def generate(self) -> float:
        return lib().po_mt_generate(ptr(self.buf))

    def generate_between(self, lo, hi) -> float:
        return lib().po_mt_generate_between(ptr(self.buf), lo, hi)


def scene(name: str, w: int, h: int):
    sp = np.zeros(16, dtype=SPHERE_DT)
    cfg = np.zeros(1, dtype=CAMCFG_DT)
    n = lib().po_scene(SCENES[name], w, h, ptr(sp), 16, ptr(cfg))
    assert n > 0
    return sp[:n].copy(), cfg


def synthetic_scene(n: int, w: int, h: int, gen_seed: int = 42):
    sp = np.zeros(n, dtype=SPHERE_DT)
    cfg = np.zeros(1, dtype=CAMCFG_DT)
    assert lib().po_scene_synthetic(n, w, h, gen_seed, ptr(sp), ptr(cfg)) == n
    return sp, cfg


def camera_with_config(cfg) -> np.ndarray:
    cam = np.zeros(1, dtype=CAMERA_DT)
    lib().po_camera_with_config(ptr(np.ascontiguousarray(cfg)), ptr(cam))
    return cam


def sphere_intersect(sp, o, d) -> float:
    one = np.ascontiguousarray(np.asarray(sp).reshape(1))
    return lib().po_sphere_intersect(ptr(one), ptr(vec(o)), ptr(vec(d)))


def hit_record(sp, o, d, t) -> np.ndarray:
    out = np.zeros(10)
    one = np.ascontiguousarray(np.asarray(sp).reshape(1))
    lib().po_hit_record(ptr(one), ptr(vec(o)), ptr(vec(d)), t, ptr(out))
    return out


def get_ray(cam, s, t, rng: MT19937):
    o = np.zeros(3)
    d = np.zeros(3)
    draws = lib().po_camera_get_ray_mt(ptr(cam), s, t, ptr(rng.buf), ptr(o), ptr(d))
    return o, d, draws


def radiance_mt(spheres, o, d, rng: MT19937):
    out = np.zeros(3)
    segs = lib().po_radiance_mt(ptr(spheres), len(spheres), ptr(vec(o)), ptr(vec(d)),
                                ptr(rng.buf), ptr(out))
    return out, segs


# ---------------------------------------------------------------- renders
def render_mt(spheres, cam, W, H, samps, nsub=2, rd_value=1, rows=None, nthreads=8):
    y0, y1, ys = rows if rows is not None else (0, H, 1)
    img = np.zeros((H * W * 3,), dtype=np.float64)
    rc = lib().po_render_mt(ptr(spheres), len(spheres), ptr(cam), W, H, samps, nsub,
                            rd_value, y0, y1, ys, nthreads, ptr(img))
    assert rc == 0
    return img.reshape(H, W, 3)


def render_xs_f64(spheres, cam, W, H, samps, nsub=2, seed=0x5EED0001, rows=None, nthreads=8):
    y0, y1, ys = rows if rows is not None else (0, H, 1)
    img = np.zeros((H * W * 3,), dtype=np.float64)
    segs = np.zeros(1, dtype=np.uint64)
    rc = lib().po_render_xs_f64(ptr(spheres), len(spheres), ptr(cam), W, H, samps, nsub, seed,
                                y0, y1, ys, nthreads, ptr(img), ptr(segs))
    assert rc == 0
    return img.reshape(H, W, 3), int(segs[0])


def render_xs_f32(spheres, cam, W, H, samps, nsub=2, seed=0x5EED0001, rows=None, nthreads=8):
    y0, y1, ys = rows if rows is not None else (0, H, 1)
    img = np.zeros((H * W * 3,), dtype=np.float32)
    segs = np.zeros(1, dtype=np.uint64)
    rc = lib().po_render_xs_f32(ptr(spheres), len(spheres), ptr(cam), W, H, samps, nsub, seed,
                                y0, y1, ys, nthreads, ptr(img), ptr(segs))
    assert rc == 0
    return img.reshape(H, W, 3), int(segs[0])


def render_xs_rect(spheres, cam, W, H, samps, nsub=2, seed=0x5EED0001, cols=None, rows=None, nthreads=8,
                   f64=False):
    """Mode A/xs (f64=True) or Mode B image of the pixels x in cols = (x0, x1)
    of rows = (y0, y1, ystep), rendered in parallel over pixels (a single row
    at a large sample count uses every thread); other pixels stay 0."""
    x0, x1 = cols if cols is not None else (0, W)
    y0, y1, ys = rows if rows is not None else (0, H, 1)
    img = np.zeros((H * W * 3,), dtype=np.float64 if f64 else np.float32)
    segs = np.zeros(1, dtype=np.uint64)
    fn = lib().po_render_xs_f64_rect if f64 else lib().po_render_xs_f32_rect
    rc = fn(ptr(spheres), len(spheres), ptr(cam), W, H, samps, nsub, seed, x0, x1, y0, y1, ys, nthreads, ptr(img),
            ptr(segs))
    assert rc == 0
    return img.reshape(H, W, 3), int(segs[0])


# Mode B' flags (pt_oracle.c): each swaps one deliberate approximation of
# Mode B for the accurate fp32 operation (error decomposition only)
BV_IEEE_SQRT, BV_IEEE_DIV, BV_LIBM_TRIG, BV_RENORM, BV_FULL_SCAN, BV_LEX = 1, 2, 4, 8, 16, 32
BV_DISC_NAIVE = 64  # round 1's discriminant hb^2 - a c for small spheres (a formulation, not an approximation)
BV_NAIVE_ROOTS = 128  # small spheres' roots (-hb -+ sqrt(disc)) / a (round 4: C3 RMSE 5e-5 -> 4.5e-4, not kept)
BV_ALL = 63  # every approximation swapped for the accurate fp32 operation


class mode_b_variant:
    """Context manager: render Mode B with the given B' flags (0 = Mode B)."""

    def __init__(self, flags: int):
        self.flags = flags

    def __enter__(self):
        self.prev = lib().po_get_mode_b_variant()
        lib().po_set_mode_b_variant(self.flags)
        return self

    def __exit__(self, *exc):
        lib().po_set_mode_b_variant(self.prev)


def render_xs_f32_count(spheres, cam, W, H, samps, nsub=2, seed=0x5EED0001, rows=None, nthreads=8):
    """Mode B image, segments and the count of paths whose radiance the exact
    accumulation clips (NaN / negative / > 2^30)."""
    y0, y1, ys = rows if rows is not None else (0, H, 1)
    img = np.zeros((H * W * 3,), dtype=np.float32)
    cnt = np.zeros(2, dtype=np.uint64)
    rc = lib().po_render_xs_f32_ex(ptr(spheres), len(spheres), ptr(cam), W, H, samps, nsub, seed,
                                   y0, y1, ys, nthreads, ptr(img), ptr(cnt[:1]), ptr(cnt[1:]))
    assert rc == 0
    return img.reshape(H, W, 3), int(cnt[0]), int(cnt[1])


def sample_f32(spheres, cam, W, H, nsub, seed, x, y, sx, sy, sample):
    out = np.zeros(3, dtype=np.float32)
    segs = lib().po_sample_f32(ptr(spheres), len(spheres), ptr(cam), W, H, nsub, seed,
                               x, y, sx, sy, sample, ptr(out))
    return out, segs


def tonemap(image: np.ndarray) -> np.ndarray:
    img = np.ascontiguousarray(image, dtype=np.float64)
    out = np.zeros(img.size, dtype=np.int32)
    lib().po_tonemap(ptr(img), img.size, ptr(out))
    return out.reshape(img.shape)


def scan_layout(spheres, cam):
    """Mode B anchor axis per sphere and the linear scan order."""
    n = len(spheres)
    axis = np.zeros(max(n, 1), dtype=np.int32)
    order = np.zeros(max(n, 1), dtype=np.int32)
    assert lib().po_scan_layout(ptr(spheres), n, ptr(cam), ptr(axis), ptr(order)) == 0
    return axis[:n].tolist(), order[:n].tolist()


def anchor_axes(spheres, cam):
    return scan_layout(spheres, cam)[0]


def sincos2pi(m):
    """Mode B {cos, sin}(2 pi m / 2^24) for 24-bit integers m."""
    m = np.ascontiguousarray(m, dtype=np.uint32)
    out = np.zeros((m.size, 2), dtype=np.float32)
    lib().po_sincos2pi(ptr(m), m.size, ptr(out))
    return out


def mode_b_roots(a):
    """Mode B's scan square root and normalising reciprocal square root."""
    a = np.ascontiguousarray(a, dtype=np.float32)
    s = np.zeros_like(a)
    r = np.zeros_like(a)
    lib().po_mode_b_roots(ptr(a), a.size, ptr(s), ptr(r))
    return s, r


def mode_b_math(a, b):
    """Mode B division a / b (b > 0) and square root of a."""
    a = np.ascontiguousarray(a, dtype=np.float32)
    b = np.ascontiguousarray(b, dtype=np.float32)
    q = np.zeros_like(a)
    r = np.zeros_like(a)
    lib().po_mode_b_math(ptr(a), ptr(b), a.size, ptr(q), ptr(r))
    return q, r
