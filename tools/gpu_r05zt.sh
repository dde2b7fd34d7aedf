#!/usr/bin/env bash
# Round 5: SAH bins per axis in the BVH build (PTG_SAH_BINS 16 / 64 / 128;
# HEAD 32) -- BVH parity of b128, then same-box C5 timing with test counts.
tag=${1:-r05zt}
bash tools/gpu_bvh_ab.sh ${tag} "b128" "main b16 b64 b128" 2
