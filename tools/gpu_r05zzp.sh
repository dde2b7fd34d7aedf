#!/usr/bin/env bash
# Round 5: the linear kernel's prefetched camera ray read from LDS before
# the segment (PTG_PRE_EARLY, _pe: a path that ends starts the next without
# waiting on the read; 64 VGPRs) -- parity and accuracy tests, then same-box
# timing on the bench frame and C3.
tag=${1:-r05zzp}
mkdir -p gpurun_out
PTGPU_LIB=cpu-path-tracing_amd/build/libptgpu_pe.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 \
  --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_fast_math.py tests/test_gpu_reference.py -k "not cli" \
  > gpurun_out/${tag}_pe_tests.log 2>&1 || { echo "pe tests failed"; tail -15 gpurun_out/${tag}_pe_tests.log; exit 1; }
echo "pe: $(tail -1 gpurun_out/${tag}_pe_tests.log)"
bash tools/gpu_ab.sh ${tag} "main pe" 4 "--steps 3 --warmup 1;--workload c3 --steps 3 --warmup 1"
