#!/usr/bin/env bash
# Same-box profile A/B of library variants (PTGPU_LIB): kernel trace, SQ
# instruction mix and VALU busy passes of one workload per variant,
# summarised into gpurun_out/prof_<tag>_<variant>/ab_summary.json.
# Usage (GPU box): bash tools/prof_ab.sh <tag> "<variants>" [bench args]
set -euo pipefail
tag=$1; vars=$2; shift 2
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
for v in $vars; do
  lib=cpu-path-tracing_amd/build/libptgpu_$v.so; [ "$v" = main ] && lib=cpu-path-tracing_amd/libptgpu.so
  out=gpurun_out/prof_${tag}_$v
  mkdir -p "$out"
  BENCH=(bench.py --steps 2 --warmup 1 --cpu-baseline off "$@")
  PTGPU_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/trace" -o run --output-format csv -- python3 "${BENCH[@]}" > "$out/bench_trace.json" 2> "$out/trace.err"
  PTGPU_LIB=$lib timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAIT_INST_ANY -d "$out/sq" -o run --output-format csv -- python3 "${BENCH[@]}" > "$out/bench_sq.json" 2> "$out/sq.err"
  PTGPU_LIB=$lib timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS -d "$out/busy" -o run --output-format csv -- python3 "${BENCH[@]}" > "$out/bench_busy.json" 2> "$out/busy.err"
  python3 tools/prof_ab_summary.py "$out"
done
