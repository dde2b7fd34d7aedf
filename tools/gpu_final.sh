#!/usr/bin/env bash
# GPU box, end of a session: the three workloads' rocprofv3 profile sets
# (profiles/run_profile.sh: bench frame, C3 box_mirror, C5 10,000 spheres) and
# the default bench line with the CPU baseline.  Usage: bash tools/gpu_final.sh <tag>
set -o pipefail
tag=${1:-x}
mkdir -p gpurun_out
bash profiles/run_profile.sh "$tag" && echo "profile box ok" &&
bash profiles/run_profile.sh "${tag}_c5" --scene synthetic:10000 && echo "profile c5 ok" &&
bash profiles/run_profile.sh "${tag}_c3" --scene box_mirror && echo "profile c3 ok" &&
timeout -k 10 400 python bench.py > gpurun_out/bench_full_$tag.json 2> gpurun_out/bench_full_$tag.err && echo "bench ok"
rc=$?
tail -c 1200 gpurun_out/bench_full_$tag.json
exit $rc
