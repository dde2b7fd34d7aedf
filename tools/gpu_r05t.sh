#!/usr/bin/env bash
# Round 5: the three small spheres' records read one test ahead, the first at
# the scan's start (PTG_SMALL_PREFETCH, build/libptgpu_spf.so; exact) --
# parity, then same-box timing on the bench frame and C3.
tag=${1:-r05t}
mkdir -p gpurun_out
PTGPU_LIB=cpu-path-tracing_amd/build/libptgpu_spf.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 \
  --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_fast_math.py -k "not cli" \
  > gpurun_out/${tag}_spf_tests.log 2>&1 || { echo "spf tests failed"; tail -15 gpurun_out/${tag}_spf_tests.log; exit 1; }
echo "spf: $(tail -1 gpurun_out/${tag}_spf_tests.log)"
bash tools/gpu_ab.sh ${tag} "main spf" 3 "--steps 3 --warmup 1;--workload c3 --steps 3 --warmup 1"
