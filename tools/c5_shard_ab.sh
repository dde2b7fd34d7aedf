#!/usr/bin/env bash
# 10,000-sphere scene: 1/2/4/8-way shard times per library variant.  Usage: bash tools/c5_shard_ab.sh "<names>"
set -e
for v in $1; do
  lib=cpu-path-tracing_amd/build/libptgpu_$v.so; [ $v = main ] && lib=cpu-path-tracing_amd/libptgpu.so
  PTGPU_LIB=$lib timeout -k 10 300 python tools/shard_sim.py --scene synthetic:10000 --counts 1 2 4 8 --steps 2 > gpurun_out/c5ss_$v.json 2> gpurun_out/c5ss_$v.err
  python -c "import json;d=json.load(open('gpurun_out/c5ss_$v.json'));print('$v', {k:(v['max_ms'],v['efficiency_vs_first']) for k,v in d['shards'].items()})"
done
