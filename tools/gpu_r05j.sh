#!/usr/bin/env bash
# Round 5: Russian roulette as an integer compare and the disk draws' scale
# folded into their fma (PTG_RR_INT, build/libptgpu_rri.so; exact
# reformulations: the same decisions and values as HEAD) -- the parity and
# RMSE tests on the variant, then same-box timing on the bench frame and C3.
tag=${1:-r05j}
mkdir -p gpurun_out
PTGPU_LIB=cpu-path-tracing_amd/build/libptgpu_rri.so timeout -k 10 900 python -u -m pytest -x -q --timeout 300 \
  --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_fast_math.py tests/test_gpu_reference.py -k "not cli" \
  > gpurun_out/${tag}_rri_tests.log 2>&1 || { echo "rri tests failed"; tail -15 gpurun_out/${tag}_rri_tests.log; exit 1; }
echo "rri: $(tail -1 gpurun_out/${tag}_rri_tests.log)"
bash tools/gpu_ab.sh ${tag} "main rri" 3 "--steps 3 --warmup 1;--workload c3 --steps 3 --warmup 1"
