#!/usr/bin/env bash
# Round 5: the BVH scan's winner as its leaf-order index, turned into the
# scene index once at the scan's end (PTG_BEST_LEAF, _bl: no dependent
# scene-index load per winning candidate) -- BVH parity, then same-box C5 timing.
tag=${1:-r05zza}
bash tools/gpu_bvh_ab.sh ${tag} "bl" "main bl" 3
