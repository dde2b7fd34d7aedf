#!/usr/bin/env bash
# Same-box A/B of library variants on a linear scene (default box 1920x1080x1024).
# Usage: bash tools/box_ab.sh "<variant names>" [scene]   ("main" = in-tree libptgpu.so)
set -e
scene=${2:-box}
ARGS="--scene $scene --width 1920 --height 1080 --spp 1024 --steps 3 --warmup 1 --cpu-baseline off $AB_ARGS"  # AB_ARGS: e.g. --exact-math
for v in $1; do
  lib=cpu-path-tracing_amd/build/libptgpu_$v.so; [ $v = main ] && lib=cpu-path-tracing_amd/libptgpu.so
  PTGPU_LIB=$lib timeout -k 10 200 python bench.py $ARGS > gpurun_out/ab_${scene}_$v.json 2> gpurun_out/ab_${scene}_$v.err
  python -c "import json;d=json.load(open('gpurun_out/ab_${scene}_$v.json'));print('$scene $v', d['ms_per_step'], d['value'])"
done
