#!/usr/bin/env bash
# Round 5: LLVM AMDGPU scheduling options as library variants (the same
# source and arithmetic): gcn-max-ilp, gcn-max-memory-clause, wave priority
# (build/libptgpu_{ilp,mclause,wprio}.so) against HEAD on box, C3 and C5.
tag=${1:-r05m}
mkdir -p gpurun_out
bash tools/gpu_ab.sh ${tag} "main ilp mclause wprio" 2 "--steps 3 --warmup 1;--workload c3 --steps 3 --warmup 1;--workload c5 --steps 3 --warmup 1"
