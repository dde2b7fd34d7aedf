#!/usr/bin/env bash
# Same-box A/B of library variants on a linear-scene workload (default: the bench frame).
# Usage: bash tools/box_ab2.sh "<variants>" [bench args]   ("main" = in-tree libptgpu.so)
set -e
vars=$1; shift
for v in $vars; do
  lib=cpu-path-tracing_amd/build/libptgpu_$v.so; [ $v = main ] && lib=cpu-path-tracing_amd/libptgpu.so
  PTGPU_LIB=$lib timeout -k 10 200 python bench.py --steps 3 --warmup 1 --cpu-baseline off "$@" > gpurun_out/ab_$v.json 2> gpurun_out/ab_$v.err
  python -c "import json;d=json.load(open('gpurun_out/ab_$v.json'));print('$v', d['config']['workload'], d['ms_per_step'], d['value'])"
done
