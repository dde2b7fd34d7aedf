#!/usr/bin/env bash
# Shard times per scene and library variant.  Usage: bash tools/scene_shard_ab.sh "<scenes>" "<names>"
set -e
for sc in $1; do for v in $2; do
  lib=cpu-path-tracing_amd/build/libptgpu_$v.so; [ $v = main ] && lib=cpu-path-tracing_amd/libptgpu.so
  PTGPU_LIB=$lib timeout -k 10 300 python tools/shard_sim.py --scene $sc --counts 1 2 4 8 --steps 2 > gpurun_out/sss_${sc%%:*}_$v.json 2> gpurun_out/sss_${sc%%:*}_$v.err
  python -c "import json;d=json.load(open('gpurun_out/sss_${sc%%:*}_$v.json'));print('$sc $v', {k:(round(v['max_ms'],2),v['efficiency_vs_first']) for k,v in d['shards'].items()})"
done; done
