"""Scenes for the 4-wide BVH walk's tests (tests/test_wide_bvh_walk.py,
tests/test_gpu_parity.py): a heavily overlapping cluster whose boxes a ray
meets many of at every level, so the walk's two-entry stack overflows and the
continuation fallback (csrc/bvh_build.hpp wide_conts) runs often."""
import numpy as np

import ptgpu


def cluster_scene(n: int, w: int, h: int, seed: int = 7) -> "ptgpu.scene":
    rng = np.random.default_rng(seed)
    D, S, G = ptgpu.reflection_type.diffuse, ptgpu.reflection_type.specular, ptgpu.reflection_type.dielectric
    scn = ptgpu.scene([ptgpu.sphere(1000.0, (0.0, -1000.0, 0.0), (0.0, 0.0, 0.0), (0.5, 0.5, 0.5), D),
                       ptgpu.sphere(1.5, (0.0, 9.0, 2.0), (9.0, 9.0, 9.0), (0.8, 0.8, 0.8), D)])
    for _ in range(n - 2):
        r = float(np.exp(rng.uniform(np.log(0.05), np.log(2.5))))
        pos = (float(rng.uniform(-6.0, 6.0)), float(rng.uniform(0.0, 6.0)), float(rng.uniform(-6.0, 6.0)))
        m = rng.uniform()
        mat = D if m < 0.8 else (S if m < 0.95 else G)
        col = tuple(float(c) for c in rng.uniform(0.2, 0.95, 3))
        scn.spheres.append(ptgpu.sphere(r, pos, (0.0, 0.0, 0.0), col, mat))
    c = scn.camera_parameters
    c.position = (0.0, 4.0, 16.0)
    c.direction = (0.0, 2.0, 0.0)
    c.aspect_ratio = w / h
    c.vertical_fov_radians = 0.8
    c.aperture = 0.0
    c.focus_distance = ptgpu.length((c.position[0] - c.direction[0], c.position[1] - c.direction[1],
                                           c.position[2] - c.direction[2]))
    return scn


def dump_scene(scn, path: str) -> None:
    """tools/wide_stack_depth.cpp input: camera position, count, ptg_sphere records."""
    cam = ptgpu.camera.with_config(scn.camera_parameters)
    sp = scn.to_array()
    with open(path, "wb") as f:
        f.write(np.asarray(cam.position, np.float64).tobytes())
        f.write(np.int32(len(sp)).tobytes())
        f.write(sp.tobytes())


def huge_only_scene(n_huge: int, n_small: int, w: int, h: int, seed: int = 11) -> "ptgpu.scene":
    """More than 64 spheres of which at most a few are small: the BVH path
    with an empty tree (n_small = 0) or a one-leaf tree (n_small <= 6) under
    many huge (anchored, linearly tested) spheres."""
    rng = np.random.default_rng(seed)
    D, S = ptgpu.reflection_type.diffuse, ptgpu.reflection_type.specular
    scn = ptgpu.scene([ptgpu.sphere(1.0, (0.0, 6.0, 0.0), (12.0, 12.0, 12.0), (0.8, 0.8, 0.8), D)] if n_small else [])
    for k in range(n_huge):
        R = float(rng.uniform(1000.0, 3000.0))
        ang = 2.0 * np.pi * k / n_huge
        dist = R + float(rng.uniform(8.0, 30.0))
        pos = (dist * float(np.cos(ang)), float(rng.uniform(-20.0, 20.0)), dist * float(np.sin(ang)))
        col = tuple(float(c) for c in rng.uniform(0.2, 0.95, 3))
        emit = (0.3, 0.3, 0.3) if k % 9 == 0 else (0.0, 0.0, 0.0)
        scn.spheres.append(ptgpu.sphere(R, pos, emit, col, S if k % 5 == 0 else D))
    for k in range(max(0, n_small - 1)):
        scn.spheres.append(ptgpu.sphere(0.5 + 0.2 * k, (1.5 * k - 2.0, 0.5, 0.0), (0.0, 0.0, 0.0), (0.7, 0.3, 0.3), D))
    c = scn.camera_parameters
    c.position = (0.0, 2.0, 6.0)
    c.direction = (0.0, 1.0, 0.0)
    c.aspect_ratio = w / h
    c.vertical_fov_radians = 1.2
    c.aperture = 0.0
    c.focus_distance = ptgpu.length((0.0, 1.0, 6.0))
    return scn
