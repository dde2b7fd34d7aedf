#!/usr/bin/env bash
# GPU box: profile of the bench frame (profiles/run_profile.sh), the default
# bench line with the CPU baseline, and a 2-rank gloo rehearsal of the N > 1
# path (C4 workload, both ranks on the one GPU).  Usage: bash tools/gpu_full.sh <tag>
set -o pipefail
tag=${1:-x}
mkdir -p gpurun_out
bash profiles/run_profile.sh "$tag" && echo "profile ok" &&
timeout -k 10 400 python bench.py > gpurun_out/bench_full_$tag.json 2> gpurun_out/bench_full_$tag.err && echo "bench ok" &&
PTG_REHEARSAL=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29533 bench.py --gpus 2 --steps 1 --warmup 1 --cpu-baseline off \
    > gpurun_out/rehearse2_$tag.json 2> gpurun_out/rehearse2_$tag.err && echo "rehearsal ok"
rc=$?
tail -c 1500 gpurun_out/bench_full_$tag.json; echo; tail -c 800 gpurun_out/rehearse2_$tag.json
exit $rc
