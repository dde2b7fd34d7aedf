#!/usr/bin/env bash
# Round 5, fifth GPU pass: the vector-memory counters of HEAD's C5 kernel
# (interleaved octant layouts; compare profiles/r05_kernel_ab.txt item 1),
# and the BVH stack depth re-swept on the interleaved layouts.
tag=${1:-r05e}
mkdir -p gpurun_out
bash tools/gpu_vmem_pmc.sh ${tag}_c5 --workload c5 > gpurun_out/${tag}_vmem_c5.txt 2>&1 || { echo vmem failed; exit 1; }
tail -9 gpurun_out/${tag}_vmem_c5.txt
bash tools/gpu_bvh_ab.sh ${tag} "st2" "main st2" 2 || exit 1
