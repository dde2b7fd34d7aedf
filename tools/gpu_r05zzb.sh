#!/usr/bin/env bash
# Round 5: the shading record's reads issued first and the roulette's draw
# computed while they are in flight (PTG_SHADE_EARLY, _se; measured on the
# box scenes in round 5 at +-0.1 %) -- on C5, whose shading record is a
# global load -- BVH parity, then same-box C5 timing.
tag=${1:-r05zzb}
bash tools/gpu_bvh_ab.sh ${tag} "se" "main se" 3
