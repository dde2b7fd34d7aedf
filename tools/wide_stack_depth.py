"""Dumps a scene for tools/wide_stack_depth.cpp and runs it:
python tools/wide_stack_depth.py synthetic:10000 [rays]."""
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "cpu-path-tracing_amd")]
import ptgpu  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "synthetic:10000"
rays = sys.argv[2] if len(sys.argv) > 2 else "200000"
scn = ptgpu.make_scene(name, 1920, 1080)
cam = ptgpu.camera.with_config(scn.camera_parameters)
sp = scn.to_array()
path = "/tmp/wide_stack_scene.bin"
with open(path, "wb") as f:
    f.write(np.asarray(cam.position, np.float64).tobytes())
    f.write(np.int32(len(sp)).tobytes())
    f.write(sp.tobytes())
exe = "/tmp/wide_stack_depth"
subprocess.check_call(["g++", "-std=c++17", "-O2", "-I", os.path.join(ROOT, "include"),
                       os.path.join(ROOT, "tools", "wide_stack_depth.cpp"), "-o", exe])
subprocess.check_call([exe, path, rays] + sys.argv[3:])
