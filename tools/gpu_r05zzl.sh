#!/usr/bin/env bash
# Round 5: BVH scenes' shading records with the material and an emission
# flag packed into s0.w, the emission read only by lanes that hit an emitter
# (PTG_SHADE_PACK, _sp: two 16-B loads per hit instead of three; exact) --
# BVH parity, then same-box C5 timing.
tag=${1:-r05zzl}
bash tools/gpu_bvh_ab.sh ${tag} "sp" "main sp" 3
