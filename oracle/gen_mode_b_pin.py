#!/usr/bin/env python3
"""gen_mode_b_pin.py -- TEST INFRASTRUCTURE ONLY.

Stores the oracle's Mode B output (the fp32 restatement the GPU's exact mode
must equal bit for bit) for a few small frames in tests/golden/mode_b_pin.npz,
so that a compiler or flag change to the oracle's own build (oracle/Makefile:
-O3, -mfma on x86-64, -ffp-contract=off) cannot move the checker silently
(ADVICE r3).  Regenerate only when Mode B's arithmetic is changed on purpose.
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import pyoracle as po  # noqa: E402

CASES = [("simple", 48, 36, 8), ("box", 48, 36, 8), ("box_mirror", 48, 36, 8), ("synthetic:300", 48, 27, 4)]


def frame(name, W, H, samps):
    if name.startswith("synthetic:"):
        sp, cfg = po.synthetic_scene(int(name.split(":")[1]), W, H)
    else:
        sp, cfg = po.scene(name, W, H)
    cam = po.camera_with_config(cfg)
    img, segs = po.render_xs_f32(sp, cam, W, H, samps, 2, 0x5EED0001, nthreads=4)
    return img, segs


def main():
    out = {}
    for name, W, H, samps in CASES:
        img, segs = frame(name, W, H, samps)
        key = name.replace(":", "_")
        out[key] = img
        out[key + "_segments"] = np.uint64(segs)
    np.savez_compressed(os.path.join(os.path.dirname(HERE), "tests", "golden", "mode_b_pin.npz"), **out)


if __name__ == "__main__":
    main()
