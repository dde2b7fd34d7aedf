#!/usr/bin/env bash
# GPU-box check: gpu tests + one bench line.  Usage: bash tools/gpu_check.sh <tag> [bench args...]
tag=${1:-x}; shift || true
timeout -k 10 400 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_$tag.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_$tag.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 180 python bench.py --steps 3 --warmup 1 --cpu-baseline off "$@" > gpurun_out/bench_$tag.json 2> gpurun_out/bench_$tag.err
rc=$?; echo "bench rc=$rc"
python -c "import json;d=json.load(open('gpurun_out/bench_$tag.json'));print(d['value'], d['ms_per_step'], d['roofline'])"
exit $rc
