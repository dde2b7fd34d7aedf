#!/usr/bin/env python3
"""Summarise a profiles/run_profile.sh output directory into a small JSON
(committed under profiles/<tag>_summary.json) plus the raw kernel_stats CSV.

HBM traffic: FETCH_SIZE and WRITE_SIZE are reported by rocprofv3 in KiB per
dispatch; per MI355X_MICROARCH.md (HBM section) FETCH_SIZE reads half the bytes
of wide coalesced streams on gfx950, so the read side is doubled (upper
bound); WRITE_SIZE is taken as is.
"""
import collections
import csv
import json
import os
import shutil
import sys


def per_kernel(path, kernel_sub, pick="last"):
    """Per counter, the value of one dispatch of the timed kernel: the render
    kernel without the counting template (render_kernel<false, ...>; bench.py
    runs the counting kernel once, untimed).  pick="last": the last dispatch,
    so the first, cold one (up to 85 MB of extra reads measured) does not skew
    the steady-state per-launch figures.  pick="min": the smallest over the
    timed kernel's dispatches -- for the HBM byte counters: the kernel's
    traffic is deterministic (the image written once, the scene read), and
    one pass (r04e) reported 205 MB of WRITE_SIZE for one of two identical
    dispatches whose other read 24.3 MB, as every other pass did.  Also
    returns every dispatch's value per counter."""
    rows = list(csv.DictReader(open(path)))
    per = collections.defaultdict(list)
    for r in rows:
        name = r["Kernel_Name"]
        if kernel_sub in name and (kernel_sub != "render_kernel" or "render_kernel<false" in name):
            per[r["Counter_Name"]].append((int(r["Dispatch_Id"]), float(r["Counter_Value"])))
    if pick == "min":
        val = {k: min(v for _, v in vs) for k, vs in per.items()}
    else:
        val = {k: max(vs)[1] for k, vs in per.items()}
    return val, rows, {k: [v for _, v in sorted(vs)] for k, vs in per.items()}


def _kernel_hash():
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, "cpu-path-tracing_amd")]
    try:
        import ptgpu
        return ptgpu.kernel_source_hash()
    except Exception:  # noqa: BLE001
        return None


def _commit():
    """HEAD of the tree (None on the GPU box, which receives no .git: then
    PTG_COMMIT names it, set by the launching script)."""
    import subprocess
    c = os.environ.get("PTG_COMMIT")
    if c:
        return c
    try:
        return subprocess.check_output(["git", "rev-parse", "--short", "HEAD"], text=True,
                                       stderr=subprocess.DEVNULL).strip()
    except (OSError, subprocess.CalledProcessError):
        return None


def main(src, tag, kernel_sub="render_kernel"):
    out = {"tag": tag, "kernel": kernel_sub}
    stats = os.path.join(src, "trace", "run_kernel_stats.csv")
    ks = list(csv.DictReader(open(stats)))
    out["kernel_stats"] = [{"name": r["Name"][:90], "calls": int(r["Calls"]), "avg_ms": float(r["AverageNs"]) / 1e6,
                            "pct": float(r["Percentage"])} for r in ks[:6]]
    # the timed kernel only: bench.py's untimed counting launch (render_kernel<true, ...>) also matches
    render = [r for r in ks if kernel_sub in r["Name"] and "render_kernel<true" not in r["Name"]]
    calls = sum(int(r["Calls"]) for r in render)
    out["render_avg_ms"] = sum(float(r["TotalDurationNs"]) for r in render) / calls / 1e6
    fetch, _, fetch_all = per_kernel(os.path.join(src, "fetch", "run_counter_collection.csv"), kernel_sub, "min")
    write, _, write_all = per_kernel(os.path.join(src, "write", "run_counter_collection.csv"), kernel_sub, "min")
    sq, rows, _ = per_kernel(os.path.join(src, "sq", "run_counter_collection.csv"), kernel_sub)
    sq2p = os.path.join(src, "sq2", "run_counter_collection.csv")
    if os.path.exists(sq2p):
        sq.update(per_kernel(sq2p, kernel_sub)[0])
    fetch_b = fetch.get("FETCH_SIZE", 0.0) * 1024 * 2  # gfx950 FETCH_SIZE = 1/2 of wide-stream bytes
    write_b = write.get("WRITE_SIZE", 0.0) * 1024
    out["hbm_bytes_per_launch"] = {"fetch_x2": fetch_b, "write": write_b, "total": fetch_b + write_b,
                                   "dispatches_KiB": {"FETCH_SIZE": fetch_all.get("FETCH_SIZE"),
                                                      "WRITE_SIZE": write_all.get("WRITE_SIZE")}}
    out["sq"] = sq
    vgpr = [r for r in rows if kernel_sub in r["Kernel_Name"] and "render_kernel<true" not in r["Kernel_Name"]]
    if vgpr:
        # rocprofv3's VGPR_Count field reads 32 on gfx950 for both the linear
        # (57 VGPRs) and the BVH render kernel (64): both allocate 64 (granule
        # 8), encoded as 64/8 - 1 = 7 in the kernel descriptor, and (7 + 1) x 4
        # = 32 is that field decoded with the older granule of 4.  The
        # allocation is recorded from the code object's metadata instead
        # (tools/kernel_resources.py), the profiler field under its own name.
        out["vgpr_rocprof_field"] = int(vgpr[0]["VGPR_Count"])
        out["sgpr"] = int(vgpr[0]["SGPR_Count"])
        out["lds_bytes"] = int(vgpr[0]["LDS_Block_Size"])
    try:
        sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
        import kernel_resources
        out["vgpr_code_object"] = kernel_resources.render_kernel_vgprs()
    except Exception as e:  # noqa: BLE001 -- optional (needs /opt/rocm's llvm tools)
        out["vgpr_code_object"] = f"unavailable: {e}"
    fp32 = [sq.get(k) for k in ("SQ_INSTS_VALU_ADD_F32", "SQ_INSTS_VALU_MUL_F32", "SQ_INSTS_VALU_FMA_F32",
                                "SQ_INSTS_VALU_TRANS_F32")]
    if all(v is not None for v in fp32) and sq.get("SQ_INSTS_VALU"):
        # FP32 add/mul/fma/trans among all VALU instructions of the timed kernel
        out["valu_fp32_share"] = sum(fp32) / sq["SQ_INSTS_VALU"]
    bench = os.path.join(src, "bench_trace.json")
    if os.path.exists(bench):
        out["bench"] = json.loads(open(bench).read().strip().splitlines()[-1])
        b = out["bench"]
        samples = b["config"]["width"] * b["config"]["height"] * b["config"]["spp"]
        segs = b["roofline"]["segments_per_sample"] * samples
        if "SQ_INSTS_VALU" in sq:
            out["valu_insts_per_segment_wave_level"] = sq["SQ_INSTS_VALU"] * 64 / segs
    busyp = os.path.join(src, "busy", "run_counter_collection.csv")
    if os.path.exists(busyp):
        bz = per_kernel(busyp, kernel_sub)[0]
        out["busy"] = bz
        grbm = bz.get("GRBM_GUI_ACTIVE", 0.0)
        if grbm > 0:
            cu = 256
            # rocprofv3 sums GRBM_GUI_ACTIVE over the 8 XCDs' GRBM instances
            cyc = grbm / 8 if grbm / (out["render_avg_ms"] * 1e-3) > 4e9 else grbm
            out["derived"] = {
                "clock_GHz": cyc / (out["render_avg_ms"] * 1e-3) / 1e9,
                # rocprof's VALUBusy (counter_defs.yaml): SQ_ACTIVE_INST_VALU / CU_NUM / GRBM_GUI_ACTIVE
                "VALUBusy_pct": 100.0 * bz["SQ_ACTIVE_INST_VALU"] / cu / cyc,
                # issue view: wave64 VALU instructions x 2 cycles (SIMD-32) over the 1,024 SIMDs' cycles
                "valu_issue_pct": 100.0 * bz["SQ_INSTS_VALU"] * 2 / (4 * cu) / cyc,
                "VALUUtilization_pct": 100.0 * bz["SQ_THREAD_CYCLES_VALU"] / (bz["SQ_ACTIVE_INST_VALU"] * 64),
                "MeanOccupancyPerCU_waves": bz["SQ_WAVE_CYCLES"] / cyc / cu,
            }
    if "bench" in out and "roofline" in out["bench"]:
        # the embedded bench line ran before this summary existed, so its
        # PMC-derived fields came from the previous profile of the workload;
        # restate them from THIS profile (the run-time values kept beside)
        rf = out["bench"]["roofline"]
        rf["pmc_fields_at_run_time"] = {k: rf.get(k) for k in ("traffic", "valu_issue_pct_profiled",
                                                               "valu_fp32_share", "profile")}
        rf["traffic"] = round(fetch_b + write_b)
        if "derived" in out:
            rf["valu_issue_pct_profiled"] = round(out["derived"]["valu_issue_pct"], 1)
        if "valu_fp32_share" in out:
            rf["valu_fp32_share"] = round(out["valu_fp32_share"], 4)
        rf["profile"] = tag
    dst = os.path.join(os.path.dirname(os.path.abspath(__file__)), f"{tag}_summary.json")
    with open(dst, "w") as f:
        json.dump(out, f, indent=1)
    shutil.copy(stats, os.path.join(os.path.dirname(dst), f"{tag}_kernel_stats.csv"))
    rec = {"workload": out.get("bench", {}).get("config", {}).get("workload"), "tag": tag,
           "hbm_bytes_per_launch": round(fetch_b + write_b)}
    # which kernel the profile is of (bench.py compares the hash with its tree's)
    rec["kernel_hash"] = _kernel_hash()
    rec["commit"] = _commit()
    if "derived" in out:
        rec["valu_issue_pct"] = round(out["derived"]["valu_issue_pct"], 1)
        rec["valu_lane_utilisation_pct"] = round(out["derived"]["VALUUtilization_pct"], 1)
        rec["clock_GHz"] = round(out["derived"]["clock_GHz"], 3)
    if "valu_fp32_share" in out:
        rec["valu_fp32_share"] = round(out["valu_fp32_share"], 4)
    if "valu_insts_per_segment_wave_level" in out:
        rec["valu_insts_per_64_lane_segments"] = round(out["valu_insts_per_segment_wave_level"], 1)
    # one record per workload (bench.py load_pmc looks its workload up)
    pt = os.path.join(os.path.dirname(dst), "pmc_traffic.json")
    try:
        with open(pt) as f:
            allrec = json.load(f)
    except (OSError, ValueError):
        allrec = {}
    if "workload" in allrec:  # older single-record file
        allrec = {allrec["workload"]: allrec}
    allrec[rec["workload"]] = rec
    with open(pt, "w") as f:
        json.dump(allrec, f, indent=1)
    print(json.dumps(out, indent=1)[:3000])


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], *(sys.argv[3:4]))
