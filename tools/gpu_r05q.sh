#!/usr/bin/env bash
# Round 5: box mode's wall geometry in a table indexed by (axis, side)
# (wgeo: PTG_WALL_GEO, one LDS round trip per scan instead of two), the
# segment's depth counted before the sky branch (dep: PTG_DEPTH_EARLY), both
# (wgdep); all exact -- parity of wgdep, then same-box timing on the bench
# frame and C3.
tag=${1:-r05q}
mkdir -p gpurun_out
PTGPU_LIB=cpu-path-tracing_amd/build/libptgpu_wgdep.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 \
  --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_fast_math.py -k "not cli" \
  > gpurun_out/${tag}_wgdep_tests.log 2>&1 || { echo "wgdep tests failed"; tail -15 gpurun_out/${tag}_wgdep_tests.log; exit 1; }
echo "wgdep: $(tail -1 gpurun_out/${tag}_wgdep_tests.log)"
bash tools/gpu_ab.sh ${tag} "main wgeo dep wgdep" 3 "--steps 3 --warmup 1;--workload c3 --steps 3 --warmup 1"
