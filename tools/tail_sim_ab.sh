#!/usr/bin/env bash
# Same-box A/B of split-tail variants on the single-GPU shard simulation.
# Usage: bash tools/tail_sim_ab.sh "<variant names>" [shard_sim args]   ("main" = in-tree libptgpu.so)
names=$1; shift || true
for v in $names; do
  lib=cpu-path-tracing_amd/build/libptgpu_$v.so; [ $v = main ] && lib=cpu-path-tracing_amd/libptgpu.so
  PTGPU_LIB=$lib timeout -k 10 200 python tools/shard_sim.py "$@" > gpurun_out/tailsim_$v.json 2> gpurun_out/tailsim_$v.err || { echo "$v failed"; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/tailsim_$v.json'));print('$v', ' '.join(f\"{k}:{s['max_ms']:.2f}ms/{s['efficiency_vs_first']:.4f}\" for k,s in d['shards'].items()))"
done
