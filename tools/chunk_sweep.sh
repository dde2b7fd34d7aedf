#!/usr/bin/env bash
# Work-unit size sweep: samples per sub-pixel per unit (0 = auto).  Usage: bash tools/chunk_sweep.sh "<chunks>" [bench args...]
chunks=$1; shift || true
for c in $chunks; do
  timeout -k 10 120 python bench.py --steps 3 --warmup 1 --cpu-baseline off --chunk $c "$@" > gpurun_out/ch_$c.json 2>/dev/null || { echo "chunk $c failed"; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/ch_$c.json'));print('chunk $c', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])"
done
