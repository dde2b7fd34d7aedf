#!/usr/bin/env python3
"""Register / LDS allocation of every kernel in libptgpu.so, from the gfx950
code object's metadata (.vgpr_count, .sgpr_count, .group_segment_fixed_size,
.vgpr_spill_count) -- what the compiler allocated, independent of any
profiler field.  Extracts the .hip_fatbin section with objcopy and the gfx950
bundle with clang-offload-bundler, then reads the AMDGPU notes with
llvm-readobj (all in /opt/rocm; no GPU needed).

  python3 tools/kernel_resources.py [libptgpu.so]   -> JSON {kernel: {...}}
"""
import json
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LLVM = "/opt/rocm/lib/llvm/bin"


def resources(lib=os.path.join(ROOT, "cpu-path-tracing_amd", "libptgpu.so")):
    with tempfile.TemporaryDirectory() as d:
        fb, co = os.path.join(d, "fb.bin"), os.path.join(d, "k.co")
        subprocess.check_call(["objcopy", "-O", "binary", "--only-section=.hip_fatbin", lib, fb])
        subprocess.check_call([os.path.join(LLVM, "clang-offload-bundler"), "--unbundle", "--type=o",
                               f"--input={fb}", "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"])
        notes = subprocess.check_output([os.path.join(LLVM, "llvm-readobj"), "--notes", co], text=True)
    # amdhsa.kernels is a YAML list: each kernel's record starts with a
    # "- .agpr_count" line (keys are sorted; .args has deeper list items)
    out, cur = {}, None
    for line in notes.splitlines():
        if re.match(r"\s+- \.agpr_count:", line):
            if cur and "name" in cur:
                out[cur.pop("name")] = cur
            cur = {}
        if cur is None:
            continue
        m = re.match(r"\s+(?:- )?\.(name|vgpr_count|agpr_count|sgpr_count|vgpr_spill_count|sgpr_spill_count|"
                     r"group_segment_fixed_size|private_segment_fixed_size):\s+(\S+)", line)
        if m and not line.lstrip().startswith("- .name"):  # (an argument's .name is a list item)
            k, v = m.group(1), m.group(2)
            if k == "name":
                if line.index(".name") <= line.index(".") and "name" not in cur:
                    cur["name"] = v
            else:
                cur.setdefault(k, int(v))
    if cur and "name" in cur:
        out[cur.pop("name")] = cur
    return out


def render_kernel_vgprs(lib=None):
    """{"linear": vgprs, "bvh": vgprs} of the fast-mode timed render kernels."""
    r = resources(lib) if lib else resources()
    pick = {}
    for name, v in r.items():
        if "render_kernelILb0ELb0ELb0E" in name:
            pick["linear"] = v["vgpr_count"]
        elif "render_kernelILb0ELb1ELb0E" in name:
            pick["bvh"] = v["vgpr_count"]
    return pick


if __name__ == "__main__":
    print(json.dumps(resources(*sys.argv[1:2]), indent=1))
