#!/usr/bin/env bash
# Round 3 (arithmetic modes): the -m gpu suite, then bench lines of both modes
# for box, box_mirror and C5.  Usage: bash tools/gpu_r03_fast.sh <tag>
tag=${1:-x}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread \
    > gpurun_out/pytest_$tag.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|error" gpurun_out/pytest_$tag.log | tail -3
[ $rc -eq 0 ] || { tail -40 gpurun_out/pytest_$tag.log; exit $rc; }
for sc in box box_mirror synthetic:10000; do
  for m in "" "--exact-math"; do
    timeout -k 10 200 python bench.py --scene $sc --steps 3 --warmup 1 --cpu-baseline off $m \
        > gpurun_out/bench_${tag}_${sc}${m}.json 2>> gpurun_out/bench_$tag.err || exit 1
    python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2], sys.argv[3] or 'fast', d['ms_per_step'], d['value'], d['roofline']['frac'])" \
        gpurun_out/bench_${tag}_${sc}${m}.json $sc "$m"
  done
done
