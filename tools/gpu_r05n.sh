#!/usr/bin/env bash
# Round 5: the BVH node step's stack pop as selects for every stepping lane
# (PTG_NODE_POP_SEL, build/libptgpu_psel.so) -- BVH parity, then same-box C5
# timing against HEAD.
tag=${1:-r05n}
mkdir -p gpurun_out
bash tools/gpu_bvh_ab.sh ${tag} "psel" "main psel" 3 || exit 1
