#!/usr/bin/env bash
# Round 5: box mode's extra walls from the wall geometry table (one LDS read
# per pass instead of two; PTG_XWALL_GEO, build/libptgpu_xwg.so; exact) --
# parity and accuracy tests, then same-box timing on the bench frame and C3.
tag=${1:-r05zn}
mkdir -p gpurun_out
PTGPU_LIB=cpu-path-tracing_amd/build/libptgpu_xwg.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 \
  --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_fast_math.py tests/test_gpu_reference.py -k "not cli" \
  > gpurun_out/${tag}_xwg_tests.log 2>&1 || { echo "xwg tests failed"; tail -15 gpurun_out/${tag}_xwg_tests.log; exit 1; }
echo "xwg: $(tail -1 gpurun_out/${tag}_xwg_tests.log)"
bash tools/gpu_ab.sh ${tag} "main xwg" 3 "--steps 3 --warmup 1;--workload c3 --steps 3 --warmup 1"
