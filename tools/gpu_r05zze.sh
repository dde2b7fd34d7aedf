#!/usr/bin/env bash
# Round 5: the BVH winner as its leaf-order code with the shading records
# also stored in leaf order (PTG_BEST_LEAF + PTG_SHADE_LEAF, _bls: no scene
# index read in the leaf loop nor to shade), against the code alone (_bl) --
# BVH parity, then same-box C5 timing.
tag=${1:-r05zze}
bash tools/gpu_bvh_ab.sh ${tag} "bls" "main bl bls" 3
