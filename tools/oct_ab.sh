#!/usr/bin/env bash
# A/B of BVH layouts on the 10,000-sphere scene + tail-chunk count on 8-way shards.
set -e
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -k "synthetic or shard or split_tail or work_unit" > gpurun_out/oct_pytest.log 2>&1 || { tail -30 gpurun_out/oct_pytest.log; exit 1; }
tail -2 gpurun_out/oct_pytest.log
C5="--scene synthetic:10000 --width 1920 --height 1080 --spp 1024 --steps 2 --warmup 1 --cpu-baseline off"
for v in main oct0 main oct0; do
  lib=cpu-path-tracing_amd/build/libptgpu_$v.so; [ $v = main ] && lib=cpu-path-tracing_amd/libptgpu.so
  PTGPU_LIB=$lib timeout -k 10 200 python bench.py $C5 > gpurun_out/oct_$v.json 2> gpurun_out/oct_$v.err
  python -c "import json;d=json.load(open('gpurun_out/oct_$v.json'));r=d['roofline'];print('$v', d['ms_per_step'], d['value'], r['sphere_tests_per_segment'], r['box_tests_per_segment'])"
done
for v in main t16; do
  lib=cpu-path-tracing_amd/build/libptgpu_$v.so; [ $v = main ] && lib=cpu-path-tracing_amd/libptgpu.so
  PTGPU_LIB=$lib timeout -k 10 200 python tools/shard_sim.py --counts 1 2 4 8 --steps 3 > gpurun_out/ss2_$v.json 2> gpurun_out/ss2_$v.err
  echo "$v $(cat gpurun_out/ss2_$v.json)"
done
