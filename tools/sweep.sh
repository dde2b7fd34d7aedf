#!/usr/bin/env bash
# A/B sweep of library variants (build/libptgpu_<name>.so) on one GPU, interleaved rounds.
# Usage: bash tools/sweep.sh "<names>" [rounds] [bench args...]
names=$1; rounds=${2:-2}; shift 2 || true
for r in $(seq 1 $rounds); do
  for n in $names; do
    PTGPU_LIB=cpu-path-tracing_amd/build/libptgpu_$n.so timeout -k 10 120 python bench.py --steps 2 --warmup 1 --cpu-baseline off "$@" > gpurun_out/sw_$n.json 2>/dev/null || { echo "$n failed"; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/sw_$n.json'));print('$n', 'round $r', d['value'], d['ms_per_step'], d['roofline']['frac'])"
  done
done
