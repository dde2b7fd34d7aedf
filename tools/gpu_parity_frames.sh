#!/usr/bin/env bash
# GPU box: whole-frame parity at the BASELINE configs (tools/full_frame_parity.py).
# Usage: bash tools/gpu_parity_frames.sh <tag>
tag=${1:-x}; out=gpurun_out/parity_$tag.jsonl; : > $out
run() { timeout -k 10 1000 python tools/full_frame_parity.py --threads 16 --f64 "$@" --out gpurun_out/pf.json && cat gpurun_out/pf.json >> $out; }
run --scene simple --width 400 --height 300 --spp 64 &&
run --scene box --width 1024 --height 768 --spp 256 &&
run --scene box_mirror --width 1920 --height 1080 --spp 1024 --chunk 24 &&
run --scene synthetic:10000 --width 1920 --height 1080 --spp 1024 --row-step 1080 --chunk 1 --skip-mode-b
rc=$?; cat $out; exit $rc
