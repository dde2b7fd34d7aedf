#!/usr/bin/env bash
# Quick GPU check of HEAD: the -m gpu suite, then bench lines of the metric
# frame and of C5.  Usage (GPU box): bash tools/gpu_quick.sh <tag> [pytest -k expr]
tag=${1:-quick}; kx=${2:-}
mkdir -p gpurun_out
if [ -n "$kx" ]; then K=(-k "$kx"); else K=(); fi
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread "${K[@]}" \
    > gpurun_out/${tag}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/${tag}_pytest.log; [ $rc -eq 0 ] || exit $rc
for w in box c5; do
  a=(); [ $w = c5 ] && a=(--workload c5)
  timeout -k 10 300 python bench.py --cpu-baseline off --steps 5 --warmup 1 "${a[@]}" > gpurun_out/${tag}_bench_$w.json \
    2> gpurun_out/${tag}_bench_$w.err || { echo "bench $w failed"; tail gpurun_out/${tag}_bench_$w.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/${tag}_bench_$w.json'));print('$w', d['ms_per_step'], d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'])"
done
