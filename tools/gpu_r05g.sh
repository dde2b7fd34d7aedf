#!/usr/bin/env bash
# Round 5: the exact arithmetic mode with and without the small-sphere unroll
# (PTG_SMALL_UNROLL; r05f's exact-mode bench line read 187.6 ms against
# round 4's 183.2).
tag=${1:-r05g}
mkdir -p gpurun_out
bash tools/gpu_ab.sh ${tag} "main nosu" 3 "--exact-math --steps 3 --warmup 1;--steps 3 --warmup 1"
