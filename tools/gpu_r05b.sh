#!/usr/bin/env bash
# Round 5, second GPU pass: the -m gpu suite + bench + rehearsals on HEAD
# (tools/gpu_r05a.sh), then the C5 single-layout BVH A/B:
# parity of build/libptgpu_one.so (PTG_BVH_ONE_LAYOUT=1), same-box timing
# against HEAD, and the vector-memory counters of both.
tag=${1:-r05b}
bash tools/gpu_r05a.sh $tag || exit 1
bash tools/gpu_bvh_ab.sh ${tag} "one" "main one" 2 || exit 1
bash tools/gpu_vmem_pmc.sh ${tag}_main --workload c5 > gpurun_out/${tag}_vmem_main.txt 2>&1 || { echo vmem main failed; exit 1; }
PTGPU_LIB=cpu-path-tracing_amd/build/libptgpu_one.so bash tools/gpu_vmem_pmc.sh ${tag}_one --workload c5 \
  > gpurun_out/${tag}_vmem_one.txt 2>&1 || { echo vmem one failed; exit 1; }
tail -9 gpurun_out/${tag}_vmem_main.txt gpurun_out/${tag}_vmem_one.txt
