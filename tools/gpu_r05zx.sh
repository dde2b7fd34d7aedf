#!/usr/bin/env bash
# Round 5: the exact mode with and without PTG_BEST_IDX (the exact bench line
# on HEAD read 182.5 ms against round 5's 175.3) -- same-box timing.
tag=${1:-r05zx}
bash tools/gpu_ab.sh ${tag} "main noidx" 3 "--exact-math --steps 3 --warmup 1"
