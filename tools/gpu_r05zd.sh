#!/usr/bin/env bash
# Round 5: fast mode, small spheres: c = |e|^2 - R^2 with -R^2 folded into
# the first fma (PTG_FAST_C_FOLD, build/libptgpu_cf.so; another rounding
# order) -- fast-mode accuracy and exact parity tests, the quality rows of box
# and box_mirror against HEAD, then same-box timing on the bench frame and C3.
tag=${1:-r05zd}
mkdir -p gpurun_out
PTGPU_LIB=cpu-path-tracing_amd/build/libptgpu_cf.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 \
  --timeout-method thread -m gpu tests/test_gpu_fast_math.py tests/test_gpu_reference.py tests/test_gpu_parity.py \
  -k "box or simple or C1 or C2 or C3" > gpurun_out/${tag}_cf_tests.log 2>&1 \
  || { echo "cf tests failed"; tail -15 gpurun_out/${tag}_cf_tests.log; exit 1; }
echo "cf: $(tail -1 gpurun_out/${tag}_cf_tests.log)"
for sc in box box_mirror; do
  timeout -k 10 600 python tools/quality_ab.py --scene $sc cpu-path-tracing_amd/libptgpu.so cpu-path-tracing_amd/build/libptgpu_cf.so \
    > gpurun_out/${tag}_quality_$sc.txt 2>&1 || { echo quality $sc failed; tail gpurun_out/${tag}_quality_$sc.txt; exit 1; }
  cat gpurun_out/${tag}_quality_$sc.txt
done
bash tools/gpu_ab.sh ${tag} "main cf" 3 "--steps 3 --warmup 1;--workload c3 --steps 3 --warmup 1"
