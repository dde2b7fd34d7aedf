#!/usr/bin/env bash
# C2 (box 1024x768x256 spp) per library variant.  Usage: bash tools/c2_ab.sh "<names>"
set -e
for v in $1; do
  lib=cpu-path-tracing_amd/build/libptgpu_$v.so; [ $v = main ] && lib=cpu-path-tracing_amd/libptgpu.so
  PTGPU_LIB=$lib timeout -k 10 120 python bench.py --width 1024 --height 768 --spp 256 --steps 10 --warmup 2 --cpu-baseline off > gpurun_out/c2_$v.json 2>/dev/null
  python -c "import json;d=json.load(open('gpurun_out/c2_$v.json'));print('$v', d['ms_per_step'], d['value'])"
done
