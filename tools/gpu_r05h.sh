#!/usr/bin/env bash
# Round 5: the fast mode's small-sphere near root as (hb^2 - disc)/(a qq)
# (PTG_SMALL_AC, build/libptgpu_ac.so): the fast-mode RMSE tests and the
# exact-mode parity, the bench frame's quality rows against HEAD
# (tools/quality_ab.py), then same-box timing on the bench frame and C3.
tag=${1:-r05h}
mkdir -p gpurun_out
PTGPU_LIB=cpu-path-tracing_amd/build/libptgpu_ac.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 \
  --timeout-method thread -m gpu tests/test_gpu_fast_math.py tests/test_gpu_reference.py tests/test_gpu_parity.py \
  -k "box or simple or C1 or C2 or C3" > gpurun_out/${tag}_ac_tests.log 2>&1 \
  || { echo "ac tests failed"; tail -15 gpurun_out/${tag}_ac_tests.log; exit 1; }
echo "ac: $(tail -1 gpurun_out/${tag}_ac_tests.log)"
timeout -k 10 600 python tools/quality_ab.py cpu-path-tracing_amd/libptgpu.so cpu-path-tracing_amd/build/libptgpu_ac.so \
  > gpurun_out/${tag}_quality.txt 2>&1 || { echo quality failed; tail gpurun_out/${tag}_quality.txt; exit 1; }
cat gpurun_out/${tag}_quality.txt
timeout -k 10 600 python tools/quality_ab.py --scene box_mirror cpu-path-tracing_amd/libptgpu.so cpu-path-tracing_amd/build/libptgpu_ac.so \
  > gpurun_out/${tag}_quality_c3.txt 2>&1 || { echo quality c3 failed; tail gpurun_out/${tag}_quality_c3.txt; exit 1; }
cat gpurun_out/${tag}_quality_c3.txt
bash tools/gpu_ab.sh ${tag} "main ac" 3 "--steps 3 --warmup 1;--workload c3 --steps 3 --warmup 1"
