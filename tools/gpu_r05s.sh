#!/usr/bin/env bash
# Round 5: the fast mode's division as the hardware reciprocal's product alone
# (PTG_FAST_DIV_RCP, build/libptgpu_fdiv.so; ~2 ulp instead of ~1) -- fast-mode
# accuracy tests, the box quality rows against HEAD, then same-box timing on
# the bench frame, C3 and C5.
tag=${1:-r05s}
mkdir -p gpurun_out
PTGPU_LIB=cpu-path-tracing_amd/build/libptgpu_fdiv.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 \
  --timeout-method thread -m gpu tests/test_gpu_fast_math.py tests/test_gpu_reference.py \
  > gpurun_out/${tag}_fdiv_tests.log 2>&1 || { echo "fdiv tests failed"; tail -15 gpurun_out/${tag}_fdiv_tests.log; exit 1; }
echo "fdiv: $(tail -1 gpurun_out/${tag}_fdiv_tests.log)"
timeout -k 10 600 python tools/quality_ab.py --scene box cpu-path-tracing_amd/libptgpu.so cpu-path-tracing_amd/build/libptgpu_fdiv.so \
  > gpurun_out/${tag}_quality_box.txt 2>&1 || { echo quality failed; tail gpurun_out/${tag}_quality_box.txt; exit 1; }
cat gpurun_out/${tag}_quality_box.txt
bash tools/gpu_ab.sh ${tag} "main fdiv" 3 "--steps 3 --warmup 1;--workload c3 --steps 3 --warmup 1;--workload c5 --steps 3 --warmup 1"
