#!/usr/bin/env bash
# Round 5: box-mode scan trims (all exact reformulations) -- the three small
# spheres' geometry from kernel arguments (ssg: PTG_SMALL_SGPR), the nearest
# plane as lane masks + direct table offset and need[] without the inf guard
# (kni: PTG_KN_MASKS + PTG_NEED_NOINF), both (all3): parity of all3, then
# same-box timing on the bench frame and C3.
tag=${1:-r05p}
mkdir -p gpurun_out
PTGPU_LIB=cpu-path-tracing_amd/build/libptgpu_all3.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 \
  --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_fast_math.py -k "not cli" \
  > gpurun_out/${tag}_all3_tests.log 2>&1 || { echo "all3 tests failed"; tail -15 gpurun_out/${tag}_all3_tests.log; exit 1; }
echo "all3: $(tail -1 gpurun_out/${tag}_all3_tests.log)"
bash tools/gpu_ab.sh ${tag} "main ssg kni all3" 3 "--steps 3 --warmup 1;--workload c3 --steps 3 --warmup 1"
