#!/usr/bin/env bash
# Round 3: the -m gpu suite on HEAD (unless SKIP_PYTEST=1), then whole-frame
# parity of the default (fast) arithmetic mode at C1, C2, C3 (Mode B and
# Mode A/xs on the box's CPUs).
tag=${1:-r03n}
mkdir -p gpurun_out
if [ "${SKIP_PYTEST:-0}" != 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
      > gpurun_out/pytest_$tag.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_$tag.log; [ $rc -eq 0 ] || exit $rc
fi
run() {
  FFP_MODE=fast timeout -k 10 600 python -u tools/full_frame_parity.py --scene $1 --width $2 --height $3 --spp $4 \
      --f64 --out gpurun_out/ffp_fast_$1.json > gpurun_out/ffp_fast_$1.log 2>&1 || exit 1
  tail -1 gpurun_out/ffp_fast_$1.log
}
run simple 400 300 64 && run box 1024 768 256 && run box_mirror 1920 1080 1024
