#!/usr/bin/env bash
# Round 5: every lane's second BRDF draw taken once too
# (PTG_DRAW2_MERGE, build/libptgpu_d2.so; each lane's draws keep their order
# and count, so exact) -- the exact parity and accuracy tests, then same-box
# timing on the bench frame, C3 and C5.
tag=${1:-r05zj}
mkdir -p gpurun_out
PTGPU_LIB=cpu-path-tracing_amd/build/libptgpu_d2.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 \
  --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_fast_math.py tests/test_gpu_reference.py -k "not cli" \
  > gpurun_out/${tag}_d2_tests.log 2>&1 || { echo "d2 tests failed"; tail -15 gpurun_out/${tag}_d2_tests.log; exit 1; }
echo "d2: $(tail -1 gpurun_out/${tag}_d2_tests.log)"
bash tools/gpu_ab.sh ${tag} "main d2" 3 "--steps 3 --warmup 1;--workload c3 --steps 3 --warmup 1;--workload c5 --steps 2 --warmup 1"
