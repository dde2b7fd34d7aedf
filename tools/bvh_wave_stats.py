"""BVH kernel wave-level statistics (debug variants PTG_WAVE_STATS=1/2, see
ptg_render.hip) next to the lane-level counts of the normal counting kernel,
on C5's scene at 1920x1080 with 16 spp.  GPU box: python tools/bvh_wave_stats.py
[variant ...] (default: the in-tree library, ws1, ws2; a variant named
<x>ws1 / <x>ws2 is build/libptgpu_<x>ws1.so with PTG_WAVE_STATS=1 / 2)"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if len(sys.argv) == 1 or sys.argv[1] != "--one":
    for v in sys.argv[1:] or ("lane", "ws1", "ws2"):
        env = dict(os.environ)
        if v != "lane":
            env["PTGPU_LIB"] = os.path.join(ROOT, "cpu-path-tracing_amd", "build", f"libptgpu_{v}.so")
        subprocess.check_call([sys.executable, __file__, "--one", v], env=env)
    sys.exit(0)
sys.path.insert(0, os.path.join(ROOT, "cpu-path-tracing_amd"))
import torch  # noqa: E402

import ptgpu  # noqa: E402

W, H, samps = 1920, 1080, 16
scn = ptgpu.make_scene("synthetic:10000", W, H)
cam = ptgpu.camera.with_config(scn.camera_parameters)
out = torch.zeros(H * W * 3, dtype=torch.float32, device="cuda")
cnt = torch.zeros(3, dtype=torch.int64, device="cuda")
with ptgpu.Context(scn, cam) as ctx:
    ctx.render_device(out, ptgpu.make_params(W, H, samps, flags=ptgpu.FLAG_COUNT_TESTS), cnt)
    torch.cuda.synchronize()
seg, a, b = (int(x) for x in cnt.cpu().tolist())
tag = sys.argv[2]
kind = "lane" if tag == "lane" else tag[-3:]
names = {"lane": ("sphere tests", "box tests"), "ws1": ("wave leaf-phase sphere iterations", "wave node steps"),
         "ws2": ("wave iterations that shade", "wave main-loop iterations")}[kind]
print(f"{tag}: per lane-segment: {names[0]} {a / seg:.3f}, {names[1]} {b / seg:.3f}; x64: {64 * a / seg:.2f}, {64 * b / seg:.2f}")
