#!/usr/bin/env bash
# Round 5, second GPU pass: the -m gpu suite + bench + rehearsals on HEAD
# (tools/gpu_r05a.sh), then the C5 BVH layout A/B:
# parity of the variants (build/libptgpu_<v>.so: one = PTG_BVH_ONE_LAYOUT=1,
# pad8 / pad36 = PTG_BVH_LAYOUT_PAD), same-box timing against HEAD, the
# vector-memory counters of HEAD and the single layout; then the box-scene
# small-sphere unroll (su) against HEAD on the bench frame and C3.
tag=${1:-r05b}
bash tools/gpu_r05a.sh $tag || exit 1
bash tools/gpu_bvh_ab.sh ${tag} "one pad8 pad36" "main one pad8 pad36" 2 || exit 1
bash tools/gpu_vmem_pmc.sh ${tag}_main --workload c5 > gpurun_out/${tag}_vmem_main.txt 2>&1 || { echo vmem main failed; exit 1; }
PTGPU_LIB=cpu-path-tracing_amd/build/libptgpu_one.so bash tools/gpu_vmem_pmc.sh ${tag}_one --workload c5 \
  > gpurun_out/${tag}_vmem_one.txt 2>&1 || { echo vmem one failed; exit 1; }
tail -9 gpurun_out/${tag}_vmem_main.txt gpurun_out/${tag}_vmem_one.txt
PTGPU_LIB=cpu-path-tracing_amd/build/libptgpu_su.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 \
  --timeout-method thread -m gpu tests/test_gpu_parity.py -k "box" > gpurun_out/${tag}_su_parity.log 2>&1 \
  || { echo "su parity failed"; tail -5 gpurun_out/${tag}_su_parity.log; exit 1; }
echo "su: $(tail -1 gpurun_out/${tag}_su_parity.log)"
bash tools/gpu_ab.sh ${tag}_box "main su" 3 "--steps 3 --warmup 1;--workload c3 --steps 3 --warmup 1"
