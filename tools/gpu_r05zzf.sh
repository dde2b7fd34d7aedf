#!/usr/bin/env bash
# Round 5: the BVH leaf loop without its branch on t <= tb -- every
# candidate's scene index loaded, the lex update as selects
# (PTG_LEAF_NOBRANCH, _lnb) -- BVH parity, then same-box C5 timing.
tag=${1:-r05zzf}
bash tools/gpu_bvh_ab.sh ${tag} "lnb" "main lnb" 3
