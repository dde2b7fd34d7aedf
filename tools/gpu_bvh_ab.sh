#!/usr/bin/env bash
# BVH parity tests on library variants, then a same-box C5 A/B of variants.
# Usage (GPU box): bash tools/gpu_bvh_ab.sh <tag> "<variants under test>" "<variants to time>" <rounds>
tag=$1; vt=$2; vars=$3; rounds=${4:-2}
mkdir -p gpurun_out
for v in $vt; do
  PTGPU_LIB=cpu-path-tracing_amd/build/libptgpu_$v.so timeout -k 10 400 python -u -m pytest -x -q --timeout 120 \
    --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_fast_math.py -k "bvh or synthetic or wide" \
    > gpurun_out/${tag}_${v}_parity.log 2>&1 || { echo "$v parity failed"; tail -5 gpurun_out/${tag}_${v}_parity.log; exit 1; }
  echo "$v: $(tail -1 gpurun_out/${tag}_${v}_parity.log)"
done
bash tools/gpu_ab.sh $tag "$vars" $rounds "--workload c5 --steps 3 --warmup 1"
