#!/usr/bin/env bash
# Round 3, default arithmetic mode: row subsets of C4 (every 16th row of 3840x2160 at 4096 spp)
# and C5 (every 108th row of synthetic:10000 1920x1080 at 1024 spp) against Mode B and Mode A/xs.
# (The C4 part alone takes ~10 min of the box's 16 CPUs: run the two in separate calls; C5=1 selects C5.)
mkdir -p gpurun_out
if [ "${C5:-0}" != 1 ]; then
FFP_MODE=fast timeout -k 10 700 python -u tools/full_frame_parity.py --scene box --width 3840 --height 2160 \
    --spp 4096 --f64 --row-step 16 --chunk 8 --out gpurun_out/ffp_fast_c4.json > gpurun_out/ffp_fast_c4.log 2>&1 || exit 1
tail -1 gpurun_out/ffp_fast_c4.log
exit 0
fi
FFP_MODE=fast timeout -k 10 700 python -u tools/full_frame_parity.py --scene synthetic:10000 --width 1920 --height 1080 \
    --spp 1024 --f64 --row-step 108 --chunk 1 --out gpurun_out/ffp_fast_c5.json > gpurun_out/ffp_fast_c5.log 2>&1 || exit 1
tail -1 gpurun_out/ffp_fast_c5.log
