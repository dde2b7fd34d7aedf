"""Wave cycles per phase of the BVH kernel's main loop (debug build:
make -C cpu-path-tracing_amd variant NAME=phase DEFS=-DPTG_BLOCK_STATS=2), on
C5's scene at 1920x1080 with 16 spp.  Run on the GPU box:
python tools/phase_times.py [variant ...]"""
import ctypes as C
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if len(sys.argv) == 1 or sys.argv[1] != "--one":
    for v in sys.argv[1:] or ("phase",):
        env = dict(os.environ, PTGPU_LIB=os.path.join(ROOT, "cpu-path-tracing_amd", "build", f"libptgpu_{v}.so"))
        subprocess.check_call([sys.executable, __file__, "--one", v], env=env)
    sys.exit(0)
sys.path.insert(0, os.path.join(ROOT, "cpu-path-tracing_amd"))
import torch  # noqa: E402

import ptgpu  # noqa: E402

NAMES = ["scan_start", "node_steps", "leaf_phases", "shade", "refill", "loop_control"]
W, H, samps = 1920, 1080, 16
scene = os.environ.get("PHASE_SCENE", "synthetic:10000")  # a linear scene needs PTG_BLOCK_STATS=3 (scan in slot 0)
if not scene.startswith("synthetic"):
    NAMES[0] = "scan"
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
cyc = [st[8 + k] for k in range(6)]
tot = sum(cyc)
lane_segs = int(segs.item())
print(sys.argv[2], scene, "wave cycles per 64 lane-segments:",
      " ".join(f"{n} {64 * c / lane_segs:.0f} ({100 * c / tot:.1f} %)" for n, c in zip(NAMES, cyc)))
if not scene.startswith("synthetic"):  # PTG_BLOCK_STATS=3: the diffuse/dielectric block inside shade
    print(f"  of which the diffuse/dielectric block: {64 * st[14] / lane_segs:.0f} ({100 * st[14] / tot:.1f} %)")
    print(f"  box mode's extra-wall block (in scan): {64 * st[15] / lane_segs:.0f} ({100 * st[15] / tot:.1f} %)")
if not scene.startswith("synthetic") and hasattr(ptgpu.lib(), "ptg_debug_stats2_"):
    s2 = (C.c_ulonglong * 16)()
    # (the refill sub-phases were accumulated by the same render; read them now)
    ptgpu.lib().ptg_debug_stats2_(s2)
    nb = max(1, s2[0])
    print(f"  refill batches {s2[0]} ({64 * s2[0] / lane_segs:.3f} per 64 lane-segments): per batch flush+park "
          f"{s2[1] / nb:.0f}, camera rays {s2[2] / nb:.0f}, begin/store {s2[3] / nb:.0f} wave cycles; per 64 "
          f"lane-segments {64 * s2[1] / lane_segs:.0f} / {64 * s2[2] / lane_segs:.0f} / {64 * s2[3] / lane_segs:.0f}")
