#!/usr/bin/env python3
"""gen_ref_paths.py -- TEST INFRASTRUCTURE ONLY.

Generates the path-level golden fixtures of SURVEY.md 8(c) from the
REFERENCE's own src/main.cpp:27-197 compiled by oracle/Makefile into
_ref/libref_main.so (see ref_main_capi.cpp; binding pyref.py).  Run in the
container that has /root/reference (`make -C oracle golden-paths`); the outputs
are data and are committed under tests/golden/:

  ref_brdf_<scene>.json  fixture 5: diffuse_ray / specular_ray / dielectric_ray
                         (main.cpp:44-97) on hit records of every sphere of the
                         scene -- front faces, back faces (rays from inside),
                         grazing rays -- with the draws consumed and the next
                         draw; covers total internal reflection, the Fresnel
                         reflection and refraction branches (main.cpp:80-96).
  ref_paths.npz          fixture 6: 4,096 seeded camera paths per scene:
                         mt19937(seed0 + k) -> s, t, get_ray, radiance
                         (main.cpp:104-158): value, draws consumed, next draw.
  ref_images.npz         fixture 7: a 64x48 image at 16 spp per scene from the
                         reference row loop (render_subpixel, main.cpp:179-197)
                         with the reference's per-row seeding
                         mt19937(RD * (unsigned short)(y^3)) (main.cpp:222-223),
                         RD standing in for std::random_device{}().
  ref_stats.npz          fixture 8: per-pixel mean and variance (ddof 1) over R
                         independently seeded reference renders at 64x48x4096
                         spp (row seeds drawn from numpy's PCG64(run)), for the
                         statistical tie of the counter RNG to the reference's
                         estimator.

The scenes and cameras come from the oracle (po.scene / po_camera_with_config),
which tests/test_oracle_golden.py pins bit for bit to the reference's scene
headers and camera.cpp.  Sphere hit parameters t come from po_sphere_intersect
(pinned to sphere.cpp the same way); every output is the reference's.
"""
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import pyoracle as po  # noqa: E402
import pyref as pr  # noqa: E402

OUT = os.path.join(os.path.dirname(HERE), "tests", "golden")
SCENES = ("box", "box_mirror", "simple")
PATH_SEED0 = 20240917
N_PATHS = 4096
IMG_W, IMG_H, IMG_SAMPS, IMG_RD = 64, 48, 4, 2654435769
STAT_W, STAT_H, STAT_SAMPS, STAT_RUNS = 64, 48, 1024, 16


def scene(name, W, H):
    sp, cfg = po.scene(name, W, H)
    return sp, po.camera_with_config(cfg)


def gen_brdf(name, threads):
    """Fixture 5: hit records on every sphere, all three samplers."""
    sp, cam = scene(name, IMG_W, IMG_H)
    rng = np.random.default_rng(5 + SCENES.index(name))
    recs = []
    cats = {"tir": 0, "fresnel_reflect": 0, "refract": 0}
    for i, s in enumerate(sp):
        c = np.array(s["position"])
        R = float(s["radius"])
        rays = []
        huge = R > 1e3
        # front faces: from the scene's interior region toward the sphere
        for _ in range(16):
            o = rng.uniform([-0.35, -0.35, -1.3], [0.35, 0.35, 1.5]) if name != "simple" else \
                rng.uniform([-2.5, 0.2, -0.5], [2.5, 2.5, 2.0])
            if huge:  # toward the wall: the direction to its centre, jittered
                d = (c - o) / np.linalg.norm(c - o) + rng.normal(0, 0.3, 3)
            else:
                tgt = c + R * rng.normal(0, 1, 3) / 2.0
                d = tgt - o
            rays.append((o, d * rng.uniform(0.5, 2.0)))
        # back faces: from inside the sphere (small spheres only; the walls'
        # interiors are 1e6 wide and their back faces are never reached)
        if not huge:
            for _ in range(16):
                o = c + rng.uniform(-0.5, 0.5, 3) * R
                d = rng.normal(0, 1, 3)
                rays.append((o, d * rng.uniform(0.5, 2.0)))
            # grazing: nearly tangent rays skimming the surface from outside
            for _ in range(4):
                n0 = rng.normal(0, 1, 3)
                n0 /= np.linalg.norm(n0)
                tang = np.cross(n0, rng.normal(0, 1, 3))
                tang /= np.linalg.norm(tang)
                o = c + n0 * R * 1.0005 - tang * 2 * R
                rays.append((o, tang))
        for o, d in rays:
            t = po.sphere_intersect(s, o, d)
            if not t > 0:
                continue
            for kind in ("diffuse", "specular", "dielectric"):
                seed = int(rng.integers(0, 2**32))
                ro, rd, draws, nxt = pr.brdf(kind, s, o, d, t, seed)
                rec = {"sphere": i, "kind": kind, "o": list(map(float, o)), "d": list(map(float, d)), "t": t,
                       "seed": seed, "ro": list(map(float, ro)), "rd": list(map(float, rd)), "draws": draws,
                       "next": nxt}
                if kind == "dielectric":
                    spec = pr.brdf("specular", s, o, d, t, seed)[1]
                    reflected = bool(np.array_equal(rd, spec))
                    cat = "fresnel_reflect" if draws == 2 else ("tir" if reflected else "refract")
                    rec["branch"] = cat
                    cats[cat] += 1
                recs.append(rec)
    return {"scene": name, "w": IMG_W, "h": IMG_H, "records": recs, "branches": cats,
            "generator": "oracle/gen_ref_paths.py (reference main.cpp:44-97 via _ref/libref_main.so)"}


def main():
    threads = int(os.environ.get("GEN_THREADS", os.cpu_count() or 8))
    os.makedirs(OUT, exist_ok=True)
    # fixture 5
    for name in SCENES:
        doc = gen_brdf(name, threads)
        with open(os.path.join(OUT, f"ref_brdf_{name}.json"), "w") as f:
            json.dump(doc, f, separators=(",", ":"))
        print(f"brdf {name}: {len(doc['records'])} records, dielectric branches {doc['branches']}")
    # fixture 6
    arrays = {}
    for name in SCENES:
        sp, cam = scene(name, IMG_W, IMG_H)
        rays, vals, draws, nxt = pr.paths(sp, cam, PATH_SEED0, N_PATHS, threads)
        arrays[f"{name}_value"] = vals
        arrays[f"{name}_draws"] = draws
        arrays[f"{name}_next"] = nxt
        arrays[f"{name}_ray"] = rays
        print(f"paths {name}: mean draws {draws.mean():.2f}, nonzero {np.mean(vals.max(1) > 0):.3f}")
    np.savez_compressed(os.path.join(OUT, "ref_paths.npz"), seed0=np.uint32(PATH_SEED0), w=IMG_W, h=IMG_H,
                        **arrays)
    # fixture 7
    imgs = {}
    for name in SCENES:
        sp, cam = scene(name, IMG_W, IMG_H)
        seeds = pr.reference_row_seeds(IMG_H, IMG_RD)
        imgs[name] = pr.render_rows(sp, cam, IMG_W, IMG_H, IMG_SAMPS, 2, seeds, nthreads=threads)
    np.savez_compressed(os.path.join(OUT, "ref_images.npz"), w=IMG_W, h=IMG_H, samps=IMG_SAMPS, nsub=2,
                        rd_value=np.uint32(IMG_RD), **imgs)
    print("images written")
    # fixture 8
    stats = {}
    rates = {}
    for name in SCENES:
        sp, cam = scene(name, STAT_W, STAT_H)
        runs = []
        t0 = time.perf_counter()
        for r in range(STAT_RUNS):
            seeds = np.random.default_rng(1000 + r).integers(1, 2**32, size=STAT_H, dtype=np.uint64)
            runs.append(pr.render_rows(sp, cam, STAT_W, STAT_H, STAT_SAMPS, 2, seeds.astype(np.uint32),
                                       nthreads=threads))
        dt = time.perf_counter() - t0
        runs = np.stack(runs)
        stats[f"{name}_mean"] = runs.mean(0)
        stats[f"{name}_var"] = runs.var(0, ddof=1)
        rates[name] = STAT_RUNS * STAT_W * STAT_H * STAT_SAMPS * 4 / dt / 1e6
        print(f"stats {name}: {dt:.1f} s on {threads} threads ({rates[name]:.3f} M samples/s), "
              f"image mean {runs.mean():.5f}")
    np.savez_compressed(os.path.join(OUT, "ref_stats.npz"), w=STAT_W, h=STAT_H, samps=STAT_SAMPS, nsub=2,
                        runs=STAT_RUNS, **stats)


if __name__ == "__main__":
    main()
