#!/usr/bin/env bash
# Round 5: groups of <= 6 spheres split too where the SAH says so
# (PTG_SAH_LEAF_CT 2 / 4 / 8: a split's two box tests weighted 0.4 / 0.8 /
# 1.6 sphere tests) -- BVH parity of ct4, then same-box C5 timing.
tag=${1:-r05zu}
bash tools/gpu_bvh_ab.sh ${tag} "ct4" "main ct2 ct4 ct8" 2
