#!/usr/bin/env bash
# Round 5: the first two small spheres' geometry read at the scan's start,
# the third one test ahead (PTG_SMALL_PF2, _pf2; exact) -- parity and
# accuracy tests, then same-box timing on the bench frame and C3.
tag=${1:-r05zzm}
mkdir -p gpurun_out
PTGPU_LIB=cpu-path-tracing_amd/build/libptgpu_pf2.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 \
  --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_fast_math.py tests/test_gpu_reference.py -k "not cli" \
  > gpurun_out/${tag}_pf2_tests.log 2>&1 || { echo "pf2 tests failed"; tail -15 gpurun_out/${tag}_pf2_tests.log; exit 1; }
echo "pf2: $(tail -1 gpurun_out/${tag}_pf2_tests.log)"
bash tools/gpu_ab.sh ${tag} "main pf2" 4 "--steps 3 --warmup 1;--workload c3 --steps 3 --warmup 1"
