#!/usr/bin/env bash
# Fast-mode quality tests on one library variant, then a same-box A/B of
# variants on the linear-scan workloads (box, C3, C1).
# Usage (GPU box): bash tools/gpu_lin_ab.sh <tag> "<variants under test>" "<variants to time>" <rounds>
tag=$1; vt=$2; vars=$3; rounds=${4:-2}
mkdir -p gpurun_out
for v in $vt; do
  PTGPU_LIB=cpu-path-tracing_amd/build/libptgpu_$v.so timeout -k 10 500 python -u -m pytest -x -q --timeout 300 \
    --timeout-method thread -m gpu tests/test_gpu_fast_math.py tests/test_gpu_reference.py tests/test_gpu_statistical.py \
    > gpurun_out/${tag}_${v}_tests.log 2>&1 || { echo "$v tests failed"; tail -30 gpurun_out/${tag}_${v}_tests.log; exit 1; }
  echo "$v: $(tail -1 gpurun_out/${tag}_${v}_tests.log)"
done
bash tools/gpu_ab.sh $tag "$vars" $rounds "--steps 3 --warmup 1;--workload c3 --steps 3 --warmup 1;--workload c1 --steps 20 --warmup 3"
