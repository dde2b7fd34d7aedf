#!/usr/bin/env bash
# One parameterised same-box A/B runner (replaces round 5's per-experiment
# gpu_r05*.sh launchers).  Each variant's parity tests run first; a variant
# whose tests fail stops the run before anything is timed.  Then the timed
# rounds interleave variants and workloads (tools/gpu_ab.sh).
#
# Usage (GPU box):
#   bash tools/ab.sh <tag> "<variants>" <rounds> "<workload args>;<...>" [test-set]
#     variants   "main" = cpu-path-tracing_amd/libptgpu.so, x = build/libptgpu_x.so
#                (make -C cpu-path-tracing_amd variant NAME=x DEFS="-D...")
#     test-set   linear (default): parity + fast-math + reference tests
#                bvh: the BVH / synthetic subset; none: no tests
# Example: bash tools/ab.sh r06a "main bx" 3 "--steps 3 --warmup 1;--workload c3 --steps 3 --warmup 1"
tag=$1; vars=$2; rounds=${3:-2}; wls=${4:-"--steps 3 --warmup 1"}; set_=${5:-linear}
mkdir -p gpurun_out
case $set_ in
  linear) T=(tests/test_gpu_parity.py tests/test_gpu_fast_math.py tests/test_gpu_reference.py -k "not cli") ;;
  bvh) T=(tests/test_gpu_parity.py tests/test_gpu_fast_math.py -k "bvh or synthetic or wide") ;;
  none) T=() ;;
  *) echo "unknown test set $set_"; exit 2 ;;
esac
if [ ${#T[@]} -gt 0 ]; then
  for v in $vars; do
    [ $v = main ] && continue
    PTGPU_LIB=cpu-path-tracing_amd/build/libptgpu_$v.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 \
      --timeout-method thread -m gpu "${T[@]}" > gpurun_out/${tag}_${v}_tests.log 2>&1 \
      || { echo "$v tests failed"; tail -15 gpurun_out/${tag}_${v}_tests.log; exit 1; }
    echo "$v: $(tail -1 gpurun_out/${tag}_${v}_tests.log)"
  done
fi
bash tools/gpu_ab.sh "$tag" "$vars" "$rounds" "$wls"
