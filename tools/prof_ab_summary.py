"""Summary of one tools/prof_ab.sh variant directory: render_kernel time
(kernel trace), SQ counters per launch, VALU issue and lane utilisation."""
import csv
import glob
import json
import sys

out = sys.argv[1]


def per_kernel(path):
    acc, rows = {}, {}
    for r in csv.DictReader(open(path)):
        if "render_kernel<false" not in r.get("Kernel_Name", ""):
            continue
        c = r["Counter_Name"]
        acc[c] = acc.get(c, 0.0) + float(r["Counter_Value"])
        rows.setdefault(c, set()).add(r.get("Dispatch_Id", ""))
    # per dispatch (the bench's untimed counting launch, warm-up and 2 timed steps)
    return {c: v / max(1, len(rows[c])) for c, v in acc.items()}


res = {}
st = glob.glob(out + "/trace/**/*kernel_stats.csv", recursive=True)
if st:
    for r in csv.DictReader(open(st[0])):
        if "render_kernel<false" in r["Name"]:
            res["render_avg_ms"] = float(r["AverageNs"]) / 1e6
            res["calls"] = int(r["Calls"])
for p in ("sq", "busy"):
    f = glob.glob(out + f"/{p}/**/*counter_collection.csv", recursive=True)
    if f:
        res[p] = per_kernel(f[0])
b = res.get("busy", {})
if b.get("GRBM_GUI_ACTIVE"):
    cyc = b["GRBM_GUI_ACTIVE"] / 8  # summed over the 8 XCDs' GRBM instances (profiles/summarize.py)
    res["valu_issue_pct"] = 100 * b["SQ_INSTS_VALU"] * 2 / 1024 / cyc
    res["lane_util_pct"] = 100 * b["SQ_THREAD_CYCLES_VALU"] / (b["SQ_ACTIVE_INST_VALU"] * 64)
    res["occupancy_waves_per_simd"] = b["SQ_WAVE_CYCLES"] / cyc / 1024
json.dump(res, open(out + "/ab_summary.json", "w"), indent=1)
flat = {k: (round(v, 3) if isinstance(v, float) else v) for k, v in res.items() if not isinstance(v, dict)}
sq = res.get("sq", {})
print(out, json.dumps(flat), "VALU/launch %.4g WAIT_ANY %.4g WAVE_CYC %.4g" % (
    sq.get("SQ_INSTS_VALU", 0), sq.get("SQ_WAIT_INST_ANY", 0), sq.get("SQ_WAVE_CYCLES", 0)))
