#!/usr/bin/env python3
"""Fast-mode image quality of library variants on the bench frame's quality
rows (bench.py cpu_baseline's check): each variant renders the frame in its
own process (PTGPU_LIB), the oracle's Mode B (fp32) and Mode A/xs (double,
same counter RNG) rows are computed once; prints one JSON line per variant.
Usage (GPU box): python tools/quality_ab.py [--scene box] [--width W] [--height H] [--spp S] <lib.so> ...
Test infrastructure (the oracle is the checker)."""
import argparse
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "oracle"), os.path.join(ROOT, "cpu-path-tracing_amd")]

RENDER = r"""
import sys, numpy as np, ptgpu
scene, W, H, samps, out = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), sys.argv[5]
scn = ptgpu.make_scene(scene, W, H)
cam = ptgpu.camera.with_config(scn.camera_parameters)
img = np.zeros(W * H * 3)
ptgpu.render(scn, cam, img, W, H, samps, 2, ptgpu.DEFAULT_SEED)
np.save(out, img.reshape(H, W, 3))
"""


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--scene", default="box")
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--spp", type=int, default=1024)
    ap.add_argument("--rows", type=int, default=4)
    ap.add_argument("--threads", type=int, default=16)
    a = ap.parse_args()
    W, H, samps = a.width, a.height, a.spp // 4
    env = dict(os.environ, PYTHONPATH=os.path.join(ROOT, "cpu-path-tracing_amd"))
    imgs = {}
    for k, lib in enumerate(a.libs):
        out = f"/tmp/quality_ab_{k}.npy"
        subprocess.run([sys.executable, "-c", RENDER, a.scene, str(W), str(H), str(samps), out], check=True,
                       env=dict(env, PTGPU_LIB=lib), timeout=300)
        imgs[lib] = np.load(out)
    import ptgpu
    import pyoracle as po
    scn = ptgpu.make_scene(a.scene, W, H)
    cam = ptgpu.camera.with_config(scn.camera_parameters)
    sp = scn.to_array().view(po.SPHERE_DT)
    ca = cam.to_array().view(po.CAMERA_DT)
    step = max(1, H // a.rows)
    ys = np.arange(step // 2, H, step)[:a.rows]
    b = np.concatenate([po.render_xs_f32(sp, ca, W, H, samps, 2, ptgpu.DEFAULT_SEED, rows=(int(y), int(y) + 1, 1),
                                         nthreads=a.threads)[0][H - 1 - y] for y in ys]).astype(np.float64)
    m = np.concatenate([po.render_xs_f64(sp, ca, W, H, samps, 2, ptgpu.DEFAULT_SEED, rows=(int(y), int(y) + 1, 1),
                                         nthreads=a.threads)[0][H - 1 - y] for y in ys])
    for lib, img in imgs.items():
        g = np.concatenate([img[H - 1 - y] for y in ys])
        print(json.dumps({"lib": os.path.basename(lib), "scene": a.scene, "rows": [int(y) for y in ys],
                          "rmse_vs_mode_b": float(np.sqrt(((g - b) ** 2).mean())),
                          "max_abs_vs_mode_b": float(np.abs(g - b).max()),
                          "rmse_vs_mode_a_xs": float(np.sqrt(((g - m) ** 2).mean())),
                          "n_px_diff_gt_1e-2": int((np.abs(g - b).max(1) > 1e-2).sum())}), flush=True)


if __name__ == "__main__":
    main()
