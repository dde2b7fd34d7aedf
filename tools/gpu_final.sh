#!/usr/bin/env bash
# Round-end check on HEAD (GPU box): the -m gpu suite and profiles
# (tools/gpu_suite_profile.sh), then __graft_entry__.smoke() and the default
# bench line (N = 1, CPU baseline included) as the driver runs them.
# Usage: bash tools/gpu_final.sh <tag>
tag=${1:-final}
bash tools/gpu_suite_profile.sh $tag || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${tag}_smoke.log 2>&1 \
  || { echo SMOKE FAILED; tail -20 gpurun_out/${tag}_smoke.log; exit 1; }
tail -1 gpurun_out/${tag}_smoke.log
timeout -k 10 300 python bench.py > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err \
  || { echo BENCH FAILED; tail gpurun_out/${tag}_bench.err; exit 1; }
cut -c1-600 gpurun_out/${tag}_bench.json
