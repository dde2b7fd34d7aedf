#!/usr/bin/env bash
# Vector-memory pipeline counters (TA / TD / TCP) of one workload's render
# kernel, one rocprofv3 --pmc pass per group.  Usage (GPU box):
#   bash tools/gpu_vmem_pmc.sh <tag> [bench args]
tag=${1:-vmem}; shift || true
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
out=gpurun_out/vmem_$tag; mkdir -p $out
B=(bench.py --steps 1 --warmup 1 --cpu-baseline off "$@")
pass() { name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" -d $out/$name -o run --output-format csv -- python3 "${B[@]}" > $out/$name.json 2> $out/$name.err || { echo "$name failed"; tail -3 $out/$name.err; exit 1; }; }
pass a TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE
pass b TD_TD_BUSY_sum TD_TC_STALL_sum
pass c TCP_PENDING_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_TCP_LATENCY_sum
pass d TA_TOTAL_WAVEFRONTS_sum TA_FLAT_READ_WAVEFRONTS_sum
pass e TCP_TA_TCP_STATE_READ_sum TCP_TOTAL_READ_sum
python3 - "$out" <<'PY'
import csv, sys, glob
out = sys.argv[1]
c = {}
for f in glob.glob(f"{out}/*/run_counter_collection.csv"):
    last = {}
    for r in csv.DictReader(open(f)):
        if "render_kernel<false" not in r["Kernel_Name"]:
            continue
        k, d = r["Counter_Name"], int(r["Dispatch_Id"])
        if k not in last or d > last[k][0]:
            last[k] = (d, float(r["Counter_Value"]))
    c.update({k: v for k, (d, v) in last.items()})
print(c)
g = c.get("GRBM_GUI_ACTIVE", 0) / 8  # summed over the 8 XCDs' GRBMs
if g:
    print("cycles (per XCD GRBM):", g)
    print("TA busy per CU / cycles:", c.get("TA_TA_BUSY_sum", 0) / 256 / g)
    print("TD busy per CU / cycles:", c.get("TD_TD_BUSY_sum", 0) / 256 / g)
    print("TD stalled by TC per CU / cycles:", c.get("TD_TC_STALL_sum", 0) / 256 / g)
    print("TA addr stalled by TC per CU-cycle:", c["TA_ADDR_STALLED_BY_TC_CYCLES_sum"] / 256 / g)
if c.get("TCP_TA_TCP_STATE_READ_sum"):
    print("avg TCP wave latency (cycles):", c["TCP_TCP_LATENCY_sum"] / c["TCP_TA_TCP_STATE_READ_sum"])
if c.get("TA_TOTAL_WAVEFRONTS_sum"):
    print("vector-memory wave instructions per CU-cycle:", c["TA_TOTAL_WAVEFRONTS_sum"] / 256 / g)
    if c.get("TCP_TOTAL_READ_sum"):
        print("TCP reads per wave-level load (TCP_TOTAL_READ / TA_TOTAL_WAVEFRONTS):",
              c["TCP_TOTAL_READ_sum"] / c["TA_TOTAL_WAVEFRONTS_sum"])
PY
