#!/usr/bin/env bash
# Round 3: the -m gpu suite on HEAD, then whole-frame parity of the default
# (fast) arithmetic mode at C1, C2, C3 (Mode B and Mode A/xs on the box's CPUs).
tag=${1:-r03n}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/pytest_$tag.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_$tag.log; [ $rc -eq 0 ] || exit $rc
for cfg in "simple 400 300 64" "box 1024 768 256" "box_mirror 1920 1080 1024"; do
  set -- $cfg
  FFP_MODE=fast timeout -k 10 600 python -u tools/full_frame_parity.py --scene $1 --width $2 --height $3 --spp $4 \
      --f64 --out gpurun_out/ffp_fast_$1.json > gpurun_out/ffp_fast_$1.log 2>&1 || exit 1
  tail -2 gpurun_out/ffp_fast_$1.log
done
