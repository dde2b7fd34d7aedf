#!/usr/bin/env bash
# Round 5: the exact mode's bench line on HEAD, then BVH leaf size 5 / 7 / 8
# (HEAD 6) with the 128-bin SAH build -- BVH parity of lf8, same-box C5 timing.
tag=${1:-r05zw}
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --exact-math --cpu-baseline off > gpurun_out/${tag}_exact_bench.json 2>gpurun_out/${tag}_exact_bench.err \
  || { echo "exact bench failed"; tail gpurun_out/${tag}_exact_bench.err; exit 1; }
cut -c1-300 gpurun_out/${tag}_exact_bench.json
bash tools/gpu_bvh_ab.sh ${tag} "lf8" "main lf5 lf7 lf8" 2
