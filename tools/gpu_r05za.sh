#!/usr/bin/env bash
# Round 5: 48-B wide BVH nodes (PTG_BVH_Q8, build/libptgpu_q8.so: 8-bit
# planes on a per-node grid, three 16-B loads per node step instead of four;
# the box tests only cull, so the images stay bit-exact) -- BVH parity, then
# same-box C5 timing against HEAD.
tag=${1:-r05za}
mkdir -p gpurun_out
bash tools/gpu_bvh_ab.sh ${tag} "q8p" "main q8 q8p" 2 || exit 1
