#!/usr/bin/env bash
# Round 5, sixth GPU pass: the cooperative node-load microbenchmark
# (tools/coop_load_bench.hip), the single-GPU shard simulation of the bench
# frame and C5 at 1/2/4/8 shards, and one bench line per BASELINE config
# (tools/workloads.sh) on HEAD.
tag=${1:-r05f}
mkdir -p gpurun_out
hipcc --offload-arch=gfx950 -O3 -o /tmp/clb tools/coop_load_bench.hip 2>/dev/null || { echo build failed; exit 1; }
timeout -k 10 120 /tmp/clb 2000 > gpurun_out/${tag}_coop_load.txt 2>&1 || { echo clb failed; cat gpurun_out/${tag}_coop_load.txt; exit 1; }
cat gpurun_out/${tag}_coop_load.txt
timeout -k 10 300 python tools/shard_sim.py > gpurun_out/${tag}_shard_sim_box.json 2> gpurun_out/${tag}_shard_sim_box.err || { echo shard_sim failed; exit 1; }
timeout -k 10 300 python tools/shard_sim.py --scene synthetic:10000 > gpurun_out/${tag}_shard_sim_c5.json 2> gpurun_out/${tag}_shard_sim_c5.err || { echo shard_sim c5 failed; exit 1; }
tail -c 600 gpurun_out/${tag}_shard_sim_box.json; tail -c 600 gpurun_out/${tag}_shard_sim_c5.json
bash tools/workloads.sh ${tag} > gpurun_out/${tag}_workloads.txt 2>&1 || { echo workloads failed; cat gpurun_out/${tag}_workloads.txt; exit 1; }
cat gpurun_out/${tag}_workloads.txt
timeout -k 10 300 python bench.py --exact-math --cpu-baseline off > gpurun_out/${tag}_exact.json 2>/dev/null && cut -c1-300 gpurun_out/${tag}_exact.json
