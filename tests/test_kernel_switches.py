"""Compile-only builds of the kernel's remaining non-default switches
("a CPU-side compile-only build of each kept switch").

Round 6 removed every measured-and-rejected A/B branch from
csrc/ptg_render.hip; what stays are debug builds (block / wave statistics,
the per-unit trace, the analysis build with box mode assumed) and numeric
tunables of the BVH walk.  No timed kernel uses them, so nothing else
compiles them: this test builds each one's device code for gfx950 (hipcc
cross-compiles without a GPU), so a switch cannot rot silently.
"""
import concurrent.futures as cf
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "cpu-path-tracing_amd", "csrc", "ptg_render.hip")
HIPCC = "/opt/rocm/bin/hipcc"
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "-fno-slp-vectorize", "-Wall",
         "-Wno-unused-result", "--offload-device-only", "-c"]

# every non-default value a tool or an A/B record builds (tools/phase_times.py,
# tools/unit_trace.py, tools/isa_breakdown.py, profiles/r06m_*)
SWITCHES = [
    "-DPTG_BLOCK_STATS=1",
    "-DPTG_BLOCK_STATS=2",
    "-DPTG_BLOCK_STATS=3",
    "-DPTG_WAVE_STATS=1",
    "-DPTG_WAVE_STATS=2",
    "-DPTG_UNIT_TRACE=1",
    "-DPTG_ASSUME_BOX_MODE=1",
    "-DPTG_LEAF_SPLIT=0",
    "-DPTG_LEAF_SPLIT=1",
    "-DPTG_BVH_STACK=2",
    "-DPTG_BVH_HEAD_CHUNK=0",
]


def test_every_switch_is_listed():
    """the list above covers every #if on a PTG_ switch in the kernel source"""
    src = open(SRC).read()
    tested = {s.split("=")[0][2:] for s in SWITCHES}
    conds = set(re.findall(r"^#\s*if\s+(PTG_[A-Z_0-9]+)", src, re.M))
    # (PTG_BLOCK_STATS alone: the "any statistics" guard of the values above)
    assert conds <= tested, sorted(conds - tested)


def _build(defs, out):
    r = subprocess.run([HIPCC] + FLAGS + [defs, "-o", out, SRC], capture_output=True, text=True)
    return defs, r.returncode, (r.stdout + r.stderr)[-3000:]


@pytest.mark.skipif(not shutil.which(HIPCC), reason="hipcc not present")
def test_kernel_switches_compile(tmp_path):
    with cf.ThreadPoolExecutor(max_workers=4) as ex:
        futs = [ex.submit(_build, d, str(tmp_path / f"v{i}.o")) for i, d in enumerate(SWITCHES)]
        results = [f.result() for f in futs]
    bad = [(d, log) for d, rc, log in results if rc != 0]
    assert not bad, "\n\n".join(f"{d}:\n{log}" for d, log in bad)
    # (a helper only the default leaf split calls is "not needed" without it:
    # that warning is expected; any other is not)
    warned = [(d, log) for d, rc, log in results
              if re.search(r"warning: (?!function '\w+' is not needed and will not be emitted)", log)]
    assert not warned, "\n\n".join(f"{d}:\n{log}" for d, log in warned)
