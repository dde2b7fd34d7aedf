"""Wave-level execution counts of the linear kernel's blocks (debug build:
make -C cpu-path-tracing_amd variant NAME=stats DEFS=-DPTG_BLOCK_STATS=1),
per scene scan.  Run on the GPU box: python tools/block_stats.py"""
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["PTGPU_LIB"] = os.path.join(ROOT, "cpu-path-tracing_amd", "build", "libptgpu_stats.so")
sys.path.insert(0, os.path.join(ROOT, "cpu-path-tracing_amd"))
import torch  # noqa: E402

import ptgpu  # noqa: E402

NAMES = ["main_iter", "scan", "small_root", "box_extra_walls", "dg_block", "spec_block", "refill", "small_pretest"]
res = {}
for scene in ("box", "box_mirror", "simple"):
    W, H, samps = 1920, 1080, 16
    scn = ptgpu.make_scene(scene, W, H)
    cam = ptgpu.camera.with_config(scn.camera_parameters)
    out = torch.zeros(H * W * 3, dtype=torch.float32, device="cuda")
    segs = torch.zeros(1, dtype=torch.int64, device="cuda")
    st = (C.c_ulonglong * 16)()
    ptgpu.lib().ptg_debug_stats_(st)  # zero
    with ptgpu.Context(scn, cam) as ctx:
        ctx.render_device(out, ptgpu.make_params(W, H, samps), segs)
        torch.cuda.synchronize()
    ptgpu.lib().ptg_debug_stats_(st)
    lane_segs = int(segs.item())
    d = {n: st[i] for i, n in enumerate(NAMES)}
    d["lane_segments"] = lane_segs
    d["per_wave_scan"] = {n: round(st[i] / max(1, st[1]), 3) for i, n in enumerate(NAMES)}
    d["lanes_per_wave_scan"] = round(lane_segs / max(1, st[1]), 2)
    # extra box-mode walls: per wave-level scan, waves with a lane outside the room / needing a wall toward,
    # and such lanes per wave-level scan
    d["extra_walls"] = {"waves_outside": round(st[9] / max(1, st[1]), 3), "waves_need": round(st[10] / max(1, st[1]), 3),
                        "lanes_outside": round(st[11] / max(1, st[1]), 2), "lanes_need": round(st[12] / max(1, st[1]), 2),
                        # PTG_BOX_WALL_LOOP: per wave-level scan, lanes with a wall in a pass, those not culled, passes
                        # that computed the root
                        "pass_lanes": round(st[13] / max(1, st[1]), 3), "live_lanes": round(st[14] / max(1, st[1]), 3),
                        "live_passes": round(st[15] / max(1, st[1]), 3)}
    res[scene] = d
    print(scene, json.dumps(d["per_wave_scan"]), "lanes/scan", d["lanes_per_wave_scan"], json.dumps(d["extra_walls"]),
          flush=True)
json.dump(res, open(os.path.join(ROOT, "gpurun_out", "block_stats.json"), "w"), indent=1)
