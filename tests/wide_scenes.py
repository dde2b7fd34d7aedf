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
