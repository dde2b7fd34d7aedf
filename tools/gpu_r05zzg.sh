#!/usr/bin/env bash
# Round 5: a small sphere's -R^2 also in g0.w, so its test reads one 16-B
# word of its record (PTG_SMALL_G0W, _g0w; exact) -- parity and accuracy
# tests, then same-box timing on the bench frame and C3.
tag=${1:-r05zzg}
mkdir -p gpurun_out
PTGPU_LIB=cpu-path-tracing_amd/build/libptgpu_g0w.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 \
  --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_fast_math.py tests/test_gpu_reference.py -k "not cli" \
  > gpurun_out/${tag}_g0w_tests.log 2>&1 || { echo "g0w tests failed"; tail -15 gpurun_out/${tag}_g0w_tests.log; exit 1; }
echo "g0w: $(tail -1 gpurun_out/${tag}_g0w_tests.log)"
bash tools/gpu_ab.sh ${tag} "main g0w" 4 "--steps 3 --warmup 1;--workload c3 --steps 3 --warmup 1"
