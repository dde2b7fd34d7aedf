"""Static opcode-class breakdown of the linear render kernel's main loop
(VERDICT r2 next 5): compiles csrc/ptg_render.hip for gfx950 with -g (line
info only; same code), takes render_kernel<false, false>'s main loop (the
outermost loop containing the scene scan), attributes every VALU instruction
to a source region through its .loc line, and counts opcode classes per
region.  Usage: python tools/isa_breakdown.py [--asm FILE] [--defs "-D..."]"""
import collections
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "cpu-path-tracing_amd", "csrc", "ptg_render.hip")
KERNEL = os.environ.get("ISA_KERNEL", "_ZN12_GLOBAL__N_113render_kernelILb0ELb0ELb0EEEvNS_5KArgsE")  # <kCount, kBvh, kExact>: the default (fast) linear kernel


def compile_asm(defs):
    out = "/tmp/isa_breakdown.s"
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-g", "-std=c++17", "-fPIC", "-ffp-contract=off",
           "-fno-slp-vectorize", "--offload-device-only", "-S", "-o", out, SRC] + defs.split()
    subprocess.check_call(cmd, stderr=subprocess.DEVNULL)
    return out


def func_lines(path):
    """source line ranges of the functions/lambdas that matter (by signature search)"""
    src = open(path).read().splitlines()
    marks = {}
    pats = {"camera_ray": r"void camera_ray\(", "scene_scan": r"const LinRec \*scene_scan\(",
            "test_rec": r"auto test_geo = ", "test_end": r"auto test_rec = ", "box_mode": r"if \(PTG_ASSUME_BOX_MODE \|\| A\.box_mode\) \{", "axis_groups": r"\} else \{\s*$",
            "box_end": r"^        i = A\.end_ax\[2\];", "shade": r"^__device__ __forceinline__ bool shade\(const ShadeRec \*hit, float t, const float2 \*trig, f3 &o, f3 &d, f3 &T, f3 &E,$",
            "dg_block": r"if \(\(__ballot\(1\) & ~__ballot\(mat == PTG_SPECULAR\)\) != 0ull\)", "spec_block": r"if \(spec\) \{  // main.cpp:60",
            "ray_of": r"auto ray_of = ", "begin": r"auto begin = ", "flush": r"auto flush = ",
            "refill": r"auto refill = ", "main_loop": r"for \(;;\) \{"}
    for i, l in enumerate(src, 1):
        for k, p in pats.items():
            if k not in marks and re.search(p, l):
                marks[k] = i
    return marks


def region_of(f, line, m):
    if f == "pt_device.hpp":
        if 33 <= line <= 44: return "rsqrt (normalise)"
        if 52 <= line <= 68: return "sqrt (Goldschmidt)"
        if 73 <= line <= 80: return "div (t = bn/bq)"
        if 94 <= line <= 108: return "RNG keys/state"
        if 110 <= line <= 117: return "RNG draws"
        if 127 <= line <= 136: return "sin/cos table"
        return "vector math (dot/cross)"
    if f != "ptg_render.hip":
        return "other (" + f + ")"
    if m["camera_ray"] <= line < m["scene_scan"]:
        return "camera ray"
    if m["test_rec"] <= line < m["test_end"]:
        return "sphere test (test_rec)"
    if m["box_mode"] <= line < m["box_end"]:
        return "box-mode walls"
    if m["scene_scan"] <= line < m["scene_scan"] + 200:
        return "scan control"
    if m["shade"] <= line < m["dg_block"]:
        return "shade: hit, emission, RR"
    if m["dg_block"] <= line < m["spec_block"]:
        return "shade: diffuse/dielectric"
    if m["spec_block"] <= line < m["spec_block"] + 12:
        return "shade: mirror"
    if m["shade"] + 12 <= line < m["shade"] + 200:
        return "shade: other"
    if m["ray_of"] <= line < m["flush"]:
        return "path start (ray_of/begin)"
    if m["flush"] <= line < m["refill"]:
        return "path end (park/flush)"
    if m["refill"] <= line < m["refill"] + 40:
        return "refill"
    return "loop control / other"


def opclass(op):
    if op.startswith(("v_cndmask",)): return "cndmask"
    if op.startswith("v_cmp"): return "cmp"
    if op.startswith(("v_mov", "v_readfirstlane", "v_readlane", "v_writelane", "v_accvgpr")): return "mov"
    if op.startswith("v_cvt"): return "cvt"
    if re.match(r"v_(fma|fmac|mul|add|sub|subrev|max|min|mad)\w*_f32", op) or op.startswith(("v_rcp", "v_rsq", "v_sqrt", "v_fma_mix", "v_ldexp", "v_frexp", "v_exp", "v_log")):
        return "fp32"
    if op.startswith("v_"): return "int/bit"
    return None


def main():
    asm = None
    defs = ""
    if "--asm" in sys.argv:
        asm = sys.argv[sys.argv.index("--asm") + 1]
    if "--defs" in sys.argv:
        defs = sys.argv[sys.argv.index("--defs") + 1]
    asm = asm or compile_asm(defs)
    s = open(asm).read()
    files = {}
    for mm in re.finditer(r'\.file\s+(\d+)\s+"([^"]*)"(?:\s+"([^"]*)")?', s):
        files[mm.group(1)] = (mm.group(3) or mm.group(2)).split("/")[-1]
    i = s.index(KERNEL + ":")
    j = s.index(".Lfunc_end", i)
    body = s[i:j].splitlines()
    # loops: header label -> (start, end) by the last backward branch to it
    labels = {l.split(":")[0]: k for k, l in enumerate(body) if re.match(r"^\.LBB\w+:", l)}
    loops = []
    for k, l in enumerate(body):
        mm = re.search(r"s_cbranch_\w+\s+(\.LBB\w+)|s_branch\s+(\.LBB\w+)", l)
        if mm:
            tgt = mm.group(1) or mm.group(2)
            if tgt in labels and labels[tgt] < k:
                loops.append((labels[tgt], k))
    m = func_lines(SRC)
    # the main loop: the largest loop
    start, end = max(loops, key=lambda x: x[1] - x[0])
    cur = ("", 0)
    tab = collections.defaultdict(collections.Counter)
    inner = collections.Counter()
    inner_loops = [(a, b) for a, b in loops if start < a and b <= end and (a, b) != (start, end)]
    for k in range(start, end + 1):
        l = body[k].strip()
        lm = re.match(r"\.loc\s+(\d+)\s+(\d+)", l)
        if lm:
            cur = (files.get(lm.group(1), "?"), int(lm.group(2)))
            continue
        if not l or l.startswith((";", ".")):
            continue
        op = l.split()[0]
        c = opclass(op)
        if c is None:
            continue
        reg = region_of(cur[0], cur[1], m)
        tab[reg][c] += 1
        tab[reg]["VALU"] += 1
        if any(a <= k <= b for a, b in inner_loops):
            inner[reg] += 1
    classes = ["VALU", "fp32", "cndmask", "cmp", "mov", "int/bit", "cvt"]
    print(f"main loop: lines {start}-{end} of the kernel's ISA; inner loops {inner_loops}")
    print("| region | " + " | ".join(classes) + " | in inner loops |")
    print("|---|" + "---|" * (len(classes) + 1))
    tot = collections.Counter()
    for reg, c in sorted(tab.items(), key=lambda x: -x[1]["VALU"]):
        tot.update(c)
        print(f"| {reg} | " + " | ".join(str(c[k]) for k in classes) + f" | {inner[reg]} |")
    print("| total | " + " | ".join(str(tot[k]) for k in classes) + f" | {sum(inner.values())} |")


if __name__ == "__main__":
    main()
