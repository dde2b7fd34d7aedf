#!/usr/bin/env bash
# Box bench frame shards with forced unit sizes (samples per sub-pixel per unit; 0 = auto).
set -e
for c in ${1:-0 256 128 64}; do
  timeout -k 10 300 python tools/shard_sim.py --scene box --counts 1 4 8 --steps 3 --chunk $c > gpurun_out/bsc_$c.json 2> gpurun_out/bsc_$c.err
  python -c "import json;d=json.load(open('gpurun_out/bsc_$c.json'));print('chunk $c', {k:(round(v['max_ms'],2),v['efficiency_vs_first']) for k,v in d['shards'].items()})"
done
