#!/usr/bin/env bash
# GPU box: the new full-size parity tests and an informational bench line of
# the reference-arithmetic (f64) mode on the bench frame and C3.
tag=${1:-x}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "frame_size" > gpurun_out/pytest_$tag.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_$tag.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --reference-f64 --steps 2 --warmup 1 --cpu-baseline off > gpurun_out/bench_f64_$tag.json 2>&1 || exit 1
python -c "import json;d=json.load(open('gpurun_out/bench_f64_$tag.json'));print('f64 box', d['value'], d['ms_per_step'], d['roofline']['frac'])"
timeout -k 10 300 python bench.py --reference-f64 --workload c3 --steps 1 --warmup 1 --cpu-baseline off > gpurun_out/bench_f64c3_$tag.json 2>&1 || exit 1
python -c "import json;d=json.load(open('gpurun_out/bench_f64c3_$tag.json'));print('f64 c3', d['value'], d['ms_per_step'])"
