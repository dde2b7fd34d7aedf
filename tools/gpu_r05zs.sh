#!/usr/bin/env bash
# Round 5: the scan's winner as a record index relative to the sentinel
# (PTG_BEST_IDX, build/libptgpu_idx.so), the fast mode's candidate test
# without the disc < 0 compare (PTG_FAST_NO_DISC, _nod), both (_idxnod) --
# parity and accuracy tests of both, then same-box timing on the bench frame and C3.
tag=${1:-r05zs}
mkdir -p gpurun_out
PTGPU_LIB=cpu-path-tracing_amd/build/libptgpu_idxnod.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 \
  --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_fast_math.py tests/test_gpu_reference.py -k "not cli" \
  > gpurun_out/${tag}_idxnod_tests.log 2>&1 || { echo "idxnod tests failed"; tail -15 gpurun_out/${tag}_idxnod_tests.log; exit 1; }
echo "idxnod: $(tail -1 gpurun_out/${tag}_idxnod_tests.log)"
bash tools/gpu_ab.sh ${tag} "main idx nod idxnod" 3 "--steps 3 --warmup 1;--workload c3 --steps 3 --warmup 1"
