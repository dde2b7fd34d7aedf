#!/usr/bin/env bash
# The -m gpu suite on HEAD, then rocprofv3 profiles (profiles/run_profile.sh)
# of the bench frame, C3 and C5, summarised into profiles/<tag>*_summary.json.
# Usage (GPU box): bash tools/gpu_suite_profile.sh <tag> [SKIP_PYTEST=1]
tag=${1:-r04}
mkdir -p gpurun_out
if [ "${SKIP_PYTEST:-0}" != 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
      > gpurun_out/pytest_$tag.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_$tag.log; [ $rc -eq 0 ] || exit $rc
fi
bash profiles/run_profile.sh $tag || exit 1
python3 profiles/summarize.py gpurun_out/prof_$tag $tag || exit 1
bash profiles/run_profile.sh ${tag}_c3 --workload c3 || exit 1
python3 profiles/summarize.py gpurun_out/prof_${tag}_c3 ${tag}_c3 || exit 1
bash profiles/run_profile.sh ${tag}_c5 --workload c5 || exit 1
python3 profiles/summarize.py gpurun_out/prof_${tag}_c5 ${tag}_c5 || exit 1
mkdir -p gpurun_out/profiles_out && cp profiles/${tag}*_summary.json profiles/${tag}*_kernel_stats.csv profiles/pmc_traffic.json gpurun_out/profiles_out/
echo done
