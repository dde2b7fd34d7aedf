#!/usr/bin/env bash
# Round 5: every lane's first BRDF draw taken once before the samplers
# (PTG_DRAW_MERGE, build/libptgpu_dm.so; each lane's draws keep their order
# and count, so exact) -- the exact parity and accuracy tests, then same-box
# timing on the bench frame, C3 and C5.
tag=${1:-r05zi}
mkdir -p gpurun_out
PTGPU_LIB=cpu-path-tracing_amd/build/libptgpu_dm.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 \
  --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_fast_math.py tests/test_gpu_reference.py -k "not cli" \
  > gpurun_out/${tag}_dm_tests.log 2>&1 || { echo "dm tests failed"; tail -15 gpurun_out/${tag}_dm_tests.log; exit 1; }
echo "dm: $(tail -1 gpurun_out/${tag}_dm_tests.log)"
bash tools/gpu_ab.sh ${tag} "main dm" 3 "--steps 3 --warmup 1;--workload c3 --steps 3 --warmup 1;--workload c5 --steps 2 --warmup 1"
