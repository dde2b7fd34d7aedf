#!/usr/bin/env bash
# GPU box: split-tail / sharding tests, a bench line and the HBM write traffic
# (WRITE_SIZE pass) of the bench frame.  Usage: bash tools/gpu_traffic.sh <tag>
tag=${1:-x}
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/pytest_$tag.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_$tag.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --steps 5 --warmup 1 --cpu-baseline off > gpurun_out/bench_$tag.json 2> gpurun_out/bench_$tag.err || exit 1
python -c "import json;d=json.load(open('gpurun_out/bench_$tag.json'));print('box', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])"
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/w_$tag -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --cpu-baseline off > gpurun_out/bw_$tag.json 2> gpurun_out/bw_$tag.err || exit 1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/f_$tag -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --cpu-baseline off > gpurun_out/bf_$tag.json 2> gpurun_out/bf_$tag.err || exit 1
python - <<PY
import csv, collections
for k, d in (("WRITE_SIZE", "gpurun_out/w_$tag"), ("FETCH_SIZE", "gpurun_out/f_$tag")):
    rows = list(csv.DictReader(open(d + "/run_counter_collection.csv")))
    v = collections.defaultdict(list)
    for r in rows:
        v[r["Kernel_Name"][:40]].append(float(r["Counter_Value"]))
    for name, xs in v.items():
        print(k, name, "avg KiB", round(sum(xs) / len(xs), 1), "calls", len(xs))
PY
