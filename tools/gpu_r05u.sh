#!/usr/bin/env bash
# Round 5: independent work held in LDS read shadows by scheduling barriers
# (exact): the room-bound compares behind the wall record's read (ire:
# PTG_INROOM_EARLY), the roulette's draw behind the hit record's reads (she:
# PTG_SHADE_EARLY), both (ish) -- parity of ish, then same-box timing on the
# bench frame and C3.
tag=${1:-r05u}
mkdir -p gpurun_out
PTGPU_LIB=cpu-path-tracing_amd/build/libptgpu_ish.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 \
  --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_fast_math.py -k "not cli" \
  > gpurun_out/${tag}_ish_tests.log 2>&1 || { echo "ish tests failed"; tail -15 gpurun_out/${tag}_ish_tests.log; exit 1; }
echo "ish: $(tail -1 gpurun_out/${tag}_ish_tests.log)"
bash tools/gpu_ab.sh ${tag} "main ire she ish" 3 "--steps 3 --warmup 1;--workload c3 --steps 3 --warmup 1"
