"""Dumps a scene + camera for tools/packet_sim.cpp and runs it:
python tools/packet_sim.py [scene] [packets]."""
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "cpu-path-tracing_amd")]
import ptgpu  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "synthetic:10000"
W, H = 1920, 1080
scn = ptgpu.make_scene(name, W, H)
cam = ptgpu.camera.with_config(scn.camera_parameters)
path = "/tmp/packet_sim_scene.bin"
with open(path, "wb") as f:
    f.write(cam.to_array().tobytes())
    f.write(np.array([W, H, len(scn.spheres)], np.int32).tobytes())
    f.write(scn.to_array().tobytes())
exe = "/tmp/packet_sim"
subprocess.check_call(["g++", "-std=c++17", "-O2", "-I", os.path.join(ROOT, "include"),
                       os.path.join(ROOT, "tools", "packet_sim.cpp"), "-o", exe])
subprocess.check_call([exe, path] + sys.argv[2:])
