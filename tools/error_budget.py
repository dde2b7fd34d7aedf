"""Error budget of the fp32 image (Mode B = the GPU's op sequence, bit-exact)
against the reference's double-precision arithmetic with the same counter-RNG
draws (Mode A/xs), split by Mode B' variants (pt_oracle.c PO_BV_*): each swaps
one deliberate approximation for the accurate fp32 operation; "all" swaps
every one (what is left is fp32 as such); "disc_naive" restores round 1's
small-sphere discriminant hb^2 - a c.  Run from the repo root (CPU only):
    python tools/error_budget.py [out.json]
Writes profiles/r02_error_budget.json by default (DESIGN.md "error budget")."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "cpu-path-tracing_amd"), os.path.join(ROOT, "oracle")]
import ptgpu  # noqa: E402
import pyoracle as po  # noqa: E402

SEED = ptgpu.DEFAULT_SEED
NT = os.cpu_count() or 8
VARIANTS = {"mode_b": 0, "ieee_sqrt": po.BV_IEEE_SQRT, "ieee_div": po.BV_IEEE_DIV, "libm_trig": po.BV_LIBM_TRIG,
            "renormalised": po.BV_RENORM, "full_scan": po.BV_FULL_SCAN, "lex_rule": po.BV_LEX,
            "all_accurate": po.BV_ALL, "disc_naive": po.BV_DISC_NAIVE}
# name, scene, W, H, samples per sub-pixel, row step, variants
CONFIGS = [("C1 simple 400x300x64", "simple", 400, 300, 16, 1, None),
           ("box_mirror 1024x768x64", "box_mirror", 1024, 768, 16, 1, None),
           ("C2 box 1024x768x256 (48 rows)", "box", 1024, 768, 64, 16, None),
           ("C3 box_mirror 1920x1080x1024 (16 rows)", "box_mirror", 1920, 1080, 256, 67, None),
           ("C5 synthetic:10000 1920x1080x64 (2 rows)", "synthetic:10000", 1920, 1080, 16, 540,
            ["mode_b", "all_accurate", "disc_naive"])]


def main(out_path):
    res = {}
    for name, scene, W, H, samps, ystep, only in CONFIGS:
        scn = ptgpu.make_scene(scene, W, H)
        cam = ptgpu.camera.with_config(scn.camera_parameters)
        sp = scn.to_array().view(po.SPHERE_DT)
        ca = cam.to_array().view(po.CAMERA_DT)
        y0 = ystep // 2 if ystep > 1 else 0
        ys = np.arange(y0, H, ystep)
        t0 = time.time()
        a, _ = po.render_xs_f64(sp, ca, W, H, samps, 2, SEED, rows=(y0, H, ystep), nthreads=NT)
        a = a[H - 1 - ys]
        r = {"rows": len(ys), "mode_a_xs_seconds": round(time.time() - t0, 1)}
        for vname, flags in VARIANTS.items():
            if only and vname not in only:
                continue
            with po.mode_b_variant(flags):
                b, _ = po.render_xs_f32(sp, ca, W, H, samps, 2, SEED, rows=(y0, H, ystep), nthreads=NT)
            d = b[H - 1 - ys].astype(np.float64) - a
            px = np.abs(d).max(axis=2)
            r[vname] = {"rmse": float(np.sqrt((d ** 2).mean())), "max_abs": float(np.abs(d).max()),
                        "px_diff_gt_1e-3": int((px > 1e-3).sum()), "px_diff_gt_1e-2": int((px > 1e-2).sum()),
                        "pixels": int(px.size)}
            print(name, vname, "rmse %.3e" % r[vname]["rmse"], flush=True)
        res[name] = r
    with open(out_path, "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "profiles", "r02_error_budget.json"))
