#!/usr/bin/env bash
# Round 5: a Fresnel reflection's second draw taken in the Fresnel block
# instead of the mirror block (PTG_FRES_IN_BLOCK, build/libptgpu_fib.so; the
# same draw sequence per lane) -- parity and accuracy tests, then same-box
# timing on the bench frame and C3.
tag=${1:-r05zm}
mkdir -p gpurun_out
PTGPU_LIB=cpu-path-tracing_amd/build/libptgpu_fib.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 \
  --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_fast_math.py tests/test_gpu_reference.py -k "not cli" \
  > gpurun_out/${tag}_fib_tests.log 2>&1 || { echo "fib tests failed"; tail -15 gpurun_out/${tag}_fib_tests.log; exit 1; }
echo "fib: $(tail -1 gpurun_out/${tag}_fib_tests.log)"
bash tools/gpu_ab.sh ${tag} "main fib" 3 "--steps 3 --warmup 1;--workload c3 --steps 3 --warmup 1"
