#!/usr/bin/env bash
# Round 3 final on one GPU box: the -m gpu suite, the 2-rank bench rehearsal,
# then the three workloads' rocprofv3 profiles and the default bench line.
tag=${1:-r03o}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/pytest_$tag.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_$tag.log; [ $rc -eq 0 ] || exit $rc
bash tools/rehearse_multi.sh 2 || exit 1
bash tools/gpu_final.sh $tag
