#!/usr/bin/env bash
# Round 5: the BVH scan's huge-sphere records (wave-uniform addresses) read
# by scalar loads through the constant address space instead of 64-lane
# vector loads (PTG_BIG_SCALAR, _bs; C5's TD is 94.5 % busy) -- BVH parity,
# then same-box C5 timing.
tag=${1:-r05zzj}
bash tools/gpu_bvh_ab.sh ${tag} "bs" "main bs" 3
