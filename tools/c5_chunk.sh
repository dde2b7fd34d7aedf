#!/usr/bin/env bash
# 10,000-sphere scene at N=1 with forced work-unit sizes (samples per sub-pixel per unit; 0 = auto).
set -e
for c in ${1:-0 128 64 37 20 10}; do
  timeout -k 10 200 python bench.py --scene synthetic:10000 --steps 2 --warmup 1 --cpu-baseline off --chunk $c > gpurun_out/c5c_$c.json 2> gpurun_out/c5c_$c.err
  python -c "import json;d=json.load(open('gpurun_out/c5c_$c.json'));print('chunk $c', d['ms_per_step'])"
done
