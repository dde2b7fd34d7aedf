#!/usr/bin/env bash
# Round 3, default arithmetic mode: shard simulations (C4, box 1080p, C5) and the host-buffer rate
mkdir -p gpurun_out
timeout -k 10 300 python tools/shard_sim.py --scene box --width 3840 --height 2160 --spp 4096 --band-rows 1 \
    > gpurun_out/shard_sim_c4.json 2> gpurun_out/shard_sim_c4.err && tail -1 gpurun_out/shard_sim_c4.err &&
timeout -k 10 200 python tools/shard_sim.py --band-rows 1 > gpurun_out/shard_sim_box.json 2> gpurun_out/shard_sim_box.err &&
tail -1 gpurun_out/shard_sim_box.err &&
timeout -k 10 200 python tools/shard_sim.py --scene synthetic:10000 --band-rows 1 > gpurun_out/shard_sim_c5.json \
    2> gpurun_out/shard_sim_c5.err && tail -1 gpurun_out/shard_sim_c5.err &&
timeout -k 10 200 python tools/host_path_rate.py > gpurun_out/host_path_rate.txt 2>&1 && cat gpurun_out/host_path_rate.txt
