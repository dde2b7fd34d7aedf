#!/usr/bin/env bash
# Round 5: the fast mode's c fold for the BVH leaf spheres
# (PTG_FAST_C_FOLD_BVH, build/libptgpu_cfb.so) -- BVH parity and accuracy
# tests, then same-box C5 timing against HEAD.
tag=${1:-r05zg}
mkdir -p gpurun_out
PTGPU_LIB=cpu-path-tracing_amd/build/libptgpu_cfb.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 \
  --timeout-method thread -m gpu tests/test_gpu_fast_math.py tests/test_gpu_reference.py tests/test_gpu_parity.py \
  -k "C5 or bvh or synthetic or wide" > gpurun_out/${tag}_cfb_tests.log 2>&1 \
  || { echo "cfb tests failed"; tail -15 gpurun_out/${tag}_cfb_tests.log; exit 1; }
echo "cfb: $(tail -1 gpurun_out/${tag}_cfb_tests.log)"
bash tools/gpu_ab.sh ${tag} "main cfb" 3 "--workload c5 --steps 3 --warmup 1"
