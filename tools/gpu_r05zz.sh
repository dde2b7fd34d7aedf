#!/usr/bin/env bash
# Round 5: fast box mode's small spheres tested between the nearest wall's
# LDS read and its test (PTG_SMALL_FIRST, _sf), the fast mode's facing normal
# from one select and the mirror's n.d from the side's dot (PTG_FAST_NN,
# _fnn), both (_sffnn) -- parity and accuracy tests of both, then same-box
# timing on the bench frame and C3.
tag=${1:-r05zz}
mkdir -p gpurun_out
PTGPU_LIB=cpu-path-tracing_amd/build/libptgpu_sffnn.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 \
  --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_fast_math.py tests/test_gpu_reference.py -k "not cli" \
  > gpurun_out/${tag}_sffnn_tests.log 2>&1 || { echo "sffnn tests failed"; tail -15 gpurun_out/${tag}_sffnn_tests.log; exit 1; }
echo "sffnn: $(tail -1 gpurun_out/${tag}_sffnn_tests.log)"
bash tools/gpu_ab.sh ${tag} "main sf fnn sffnn" 3 "--steps 3 --warmup 1;--workload c3 --steps 3 --warmup 1"
