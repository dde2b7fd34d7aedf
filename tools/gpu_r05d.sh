#!/usr/bin/env bash
# Round 5, fourth GPU pass on HEAD (small-sphere unroll + interleaved octant
# layouts): the -m gpu suite, C5 tuning variants re-swept on the new layout
# (parity first), then the rocprofv3 profiles of the bench frame, C3 and C5
# (tools/gpu_suite_profile.sh) summarised into profiles/<tag>*.
tag=${1:-r05d}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/${tag}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/${tag}_pytest.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_bvh_ab.sh ${tag} "nt rf5 rf7 lf3 lf5 leaf5 leaf7" "main nt rf5 rf7 lf3 lf5 leaf5 leaf7" 2 || exit 1
SKIP_PYTEST=1 bash tools/gpu_suite_profile.sh ${tag} || exit 1
