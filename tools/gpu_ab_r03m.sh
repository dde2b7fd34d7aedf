#!/usr/bin/env bash
# same-box A/B (round 3, fast mode): scan latency variants; then the phase timers
bash tools/box_ab.sh "base spf su3 wsg base spf su3 wsg" && bash tools/box_ab.sh "base spf wsg" box_mirror &&
timeout -k 10 200 python tools/phase_times.py phase && PHASE_SCENE=box timeout -k 10 200 python tools/phase_times.py phase3 &&
PHASE_SCENE=box_mirror timeout -k 10 200 python tools/phase_times.py phase3 && timeout -k 10 200 python tools/bvh_wave_stats.py
# exact mode before (fb28ad0) and after the template refactor
AB_ARGS=--exact-math bash tools/box_ab.sh "old base old base"
