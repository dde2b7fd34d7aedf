#!/usr/bin/env bash
# Round 5: the roulette's colour row selected by address, one record read
# instead of two and three selects (PTG_RR_ROWSEL, _rs; exact) -- parity,
# accuracy and BVH parity tests, then same-box timing on box, C3 and C5.
tag=${1:-r05zzc}
mkdir -p gpurun_out
PTGPU_LIB=cpu-path-tracing_amd/build/libptgpu_rs.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 \
  --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_fast_math.py tests/test_gpu_reference.py -k "not cli" \
  > gpurun_out/${tag}_rs_tests.log 2>&1 || { echo "rs tests failed"; tail -15 gpurun_out/${tag}_rs_tests.log; exit 1; }
echo "rs: $(tail -1 gpurun_out/${tag}_rs_tests.log)"
bash tools/gpu_ab.sh ${tag} "main rs" 3 "--steps 3 --warmup 1;--workload c3 --steps 3 --warmup 1;--workload c5 --steps 3 --warmup 1"
