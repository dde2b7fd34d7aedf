"""Rate of the reference-shaped host call (ptg_render: scene upload, render,
device->host copy, += into the caller's double image) next to the
device-resident render (ptg_render_device into HBM, bench.py's `value`), on
the bench frame (box 1920x1080x1024 spp).  GPU box: python tools/host_path_rate.py"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cpu-path-tracing_amd"))
import torch  # noqa: E402

import ptgpu  # noqa: E402

W, H, spp, nsub = 1920, 1080, 1024, 2
samples = spp // (nsub * nsub)
scn = ptgpu.make_scene("box", W, H)
cam = ptgpu.camera.with_config(scn.camera_parameters)
img = np.zeros(W * H * 3)
ptgpu.render(scn, cam, img, W, H, samples, nsub)  # warm-up (module load, code object)
t_host = []
for _ in range(3):
    img[:] = 0.0
    t0 = time.perf_counter()
    ptgpu.render(scn, cam, img, W, H, samples, nsub)
    t_host.append(time.perf_counter() - t0)
out = torch.zeros(H * W * 3, dtype=torch.float32, device="cuda")
p = ptgpu.make_params(W, H, samples, nsub)
t_dev = []
with ptgpu.Context(scn, cam) as ctx:
    ctx.render_device(out, p)
    torch.cuda.synchronize()
    for _ in range(3):
        t0 = time.perf_counter()
        ctx.render_device(out, p)
        torch.cuda.synchronize()
        t_dev.append(time.perf_counter() - t0)
n = W * H * spp
th, td = min(t_host), min(t_dev)
print(f"ptg_render (host image, incl. context, D2H, double +=): {th * 1e3:.1f} ms = {n / th / 1e6:.0f} M samples/s")
print(f"ptg_render_device (image stays in HBM): {td * 1e3:.1f} ms = {n / td / 1e6:.0f} M samples/s")
print(f"host-side overhead: {(th - td) * 1e3:.1f} ms per frame")
