#!/usr/bin/env bash
# Round 5: the first draw's value converted once for the diffuse phi and the
# Fresnel compare (u1: PTG_U1_HOIST; exact), plus the fast mode's cos theta
# clamp as v_min_f32 (u1m: + PTG_CTH_MIN; differs only for NaN) -- parity
# and accuracy tests of u1m, then same-box timing on the bench frame and C3.
tag=${1:-r05zl}
mkdir -p gpurun_out
PTGPU_LIB=cpu-path-tracing_amd/build/libptgpu_u1m.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 \
  --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_fast_math.py tests/test_gpu_reference.py -k "not cli" \
  > gpurun_out/${tag}_u1m_tests.log 2>&1 || { echo "u1m tests failed"; tail -15 gpurun_out/${tag}_u1m_tests.log; exit 1; }
echo "u1m: $(tail -1 gpurun_out/${tag}_u1m_tests.log)"
bash tools/gpu_ab.sh ${tag} "main u1 u1m" 3 "--steps 3 --warmup 1;--workload c3 --steps 3 --warmup 1"
