#!/usr/bin/env bash
# Round 5: all three small spheres' geometry read at the scan's start
# (PTG_SMALL_PF2=2, _pf3; exact) against HEAD's first two -- parity and
# accuracy tests, then same-box timing on the bench frame and C3.
tag=${1:-r05zzn}
mkdir -p gpurun_out
PTGPU_LIB=cpu-path-tracing_amd/build/libptgpu_pf3.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 \
  --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_fast_math.py tests/test_gpu_reference.py -k "not cli" \
  > gpurun_out/${tag}_pf3_tests.log 2>&1 || { echo "pf3 tests failed"; tail -15 gpurun_out/${tag}_pf3_tests.log; exit 1; }
echo "pf3: $(tail -1 gpurun_out/${tag}_pf3_tests.log)"
bash tools/gpu_ab.sh ${tag} "main pf3" 4 "--steps 3 --warmup 1;--workload c3 --steps 3 --warmup 1"
