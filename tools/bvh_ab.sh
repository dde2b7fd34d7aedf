#!/usr/bin/env bash
# Same-box A/B of BVH library variants on the 10,000-sphere scene (C5).
# Usage: bash tools/bvh_ab.sh "<variant names>"   ("main" = in-tree libptgpu.so)
set -e
C5="--scene synthetic:10000 --width 1920 --height 1080 --spp 1024 --steps 2 --warmup 1 --cpu-baseline off"
for v in $1; do
  lib=cpu-path-tracing_amd/build/libptgpu_$v.so; [ $v = main ] && lib=cpu-path-tracing_amd/libptgpu.so
  PTGPU_LIB=$lib timeout -k 10 200 python bench.py $C5 > gpurun_out/bvh_$v.json 2> gpurun_out/bvh_$v.err
  python -c "import json;d=json.load(open('gpurun_out/bvh_$v.json'));r=d['roofline'];print('$v', d['ms_per_step'], d['value'], r['sphere_tests_per_segment'], r['box_tests_per_segment'])"
done
