#!/usr/bin/env bash
# Collects the rocprofv3 evidence behind bench.py's roofline numbers.
# Run on the GPU box from the repo root:  bash profiles/run_profile.sh <tag> [extra bench args]
# Writes gpurun_out/prof_<tag>/...; the summaries worth keeping are copied
# into profiles/ by hand (profiles/<tag>_*.csv).
#   pass 0: --kernel-trace --stats      (per-kernel durations; must agree with bench's HIP events)
#   pass 1: --pmc FETCH_SIZE            (HBM read bytes; x2 on gfx950 for wide streams, MI355X_MICROARCH.md HBM)
#   pass 2: --pmc WRITE_SIZE            (HBM write bytes)
#   pass 3: --pmc SQ instruction mix    (VALU/SALU/SMEM/LDS instruction and cycle counts)
#   pass 5: --pmc GRBM_GUI_ACTIVE + SQ  (clock, VALUBusy, VALU lane utilisation, occupancy)
set -euo pipefail
tag=${1:-r01}
shift || true
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
out=gpurun_out/prof_${tag}
mkdir -p "$out"
BENCH=(bench.py --steps 2 --warmup 1 --cpu-baseline off "$@")
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/trace" -o run --output-format csv -- python3 "${BENCH[@]}" > "$out/bench_trace.json" 2> "$out/trace.err"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d "$out/fetch" -o run --output-format csv -- python3 "${BENCH[@]}" > "$out/bench_fetch.json" 2> "$out/fetch.err"
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d "$out/write" -o run --output-format csv -- python3 "${BENCH[@]}" > "$out/bench_write.json" 2> "$out/write.err"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAIT_INST_ANY -d "$out/sq" -o run --output-format csv -- python3 "${BENCH[@]}" > "$out/bench_sq.json" 2> "$out/sq.err"
timeout -k 10 300 rocprofv3 --pmc SQ_WAIT_ANY SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_SMEM -d "$out/sq2" -o run --output-format csv -- python3 "${BENCH[@]}" > "$out/bench_sq2.json" 2> "$out/sq2.err"
timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS -d "$out/busy" -o run --output-format csv -- python3 "${BENCH[@]}" > "$out/bench_busy.json" 2> "$out/busy.err"
echo "profile $tag done"
