#!/usr/bin/env bash
# Round 5, third GPU pass: the octant layouts' placement (PTG_BVH_LAYOUT_PAD
# sweep, PTG_BVH_INTERLEAVE) on C5, and the box-scene shading split
# (PTG_DG_SPLIT) with and without the small-sphere unroll, each parity-checked
# (exact mode bit-exact) before it is timed against HEAD on the same box.
tag=${1:-r05c}
mkdir -p gpurun_out
bash tools/gpu_bvh_ab.sh ${tag} "ilv pad4 pad20 pad52 pad68 pad100 pad260" \
  "main pad36 ilv pad4 pad20 pad52 pad68 pad100 pad260" 2 || exit 1
for v in dgs dgsu; do
  PTGPU_LIB=cpu-path-tracing_amd/build/libptgpu_$v.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 \
    --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_fast_math.py -k "box or simple" \
    > gpurun_out/${tag}_${v}_parity.log 2>&1 || { echo "$v parity failed"; tail -5 gpurun_out/${tag}_${v}_parity.log; exit 1; }
  echo "$v: $(tail -1 gpurun_out/${tag}_${v}_parity.log)"
done
bash tools/gpu_ab.sh ${tag}_box "main su dgs dgsu" 2 "--steps 3 --warmup 1;--workload c3 --steps 3 --warmup 1"
