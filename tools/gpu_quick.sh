#!/usr/bin/env bash
# GPU-box check: -m gpu tests, then one bench line per listed workload.
# Usage: bash tools/gpu_quick.sh <tag> [pytest -k expr]
tag=${1:-x}; kexpr=${2:-}
mkdir -p gpurun_out
args=(tests -m gpu -x -q --timeout 120 --timeout-method thread)
[ -n "$kexpr" ] && args+=(-k "$kexpr")
timeout -k 10 600 python -u -m pytest "${args[@]}" > gpurun_out/pytest_$tag.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_$tag.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --steps 5 --warmup 1 --cpu-baseline off > gpurun_out/bench_$tag.json 2> gpurun_out/bench_$tag.err
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
python -c "import json;d=json.load(open('gpurun_out/bench_$tag.json'));print('box', d['value'], d['ms_per_step'], d['roofline']['frac'])"
timeout -k 10 200 python bench.py --scene box_mirror --steps 3 --warmup 1 --cpu-baseline off > gpurun_out/bench_${tag}_c3.json 2>> gpurun_out/bench_$tag.err
rc=$?; echo "bench c3 rc=$rc"; [ $rc -eq 0 ] || exit $rc
python -c "import json;d=json.load(open('gpurun_out/bench_${tag}_c3.json'));print('box_mirror', d['value'], d['ms_per_step'], d['roofline']['frac'])"
timeout -k 10 200 python bench.py --scene synthetic:10000 --steps 2 --warmup 1 --cpu-baseline off > gpurun_out/bench_${tag}_c5.json 2>> gpurun_out/bench_$tag.err
rc=$?; echo "bench c5 rc=$rc"; [ $rc -eq 0 ] || exit $rc
python -c "import json;d=json.load(open('gpurun_out/bench_${tag}_c5.json'));print('c5', d['value'], d['ms_per_step'], d['roofline']['frac'])"
