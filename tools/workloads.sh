#!/usr/bin/env bash
# One bench line per BASELINE.json config that fits one GPU (+ the 8-GPU configs' frames on one GPU).
# Usage: bash tools/workloads.sh <tag>
tag=${1:-w}
run() { name=$1; shift; timeout -k 10 300 python bench.py --cpu-baseline off "$@" > gpurun_out/wl_${tag}_$name.json 2>/dev/null || { echo "$name failed"; return 1; }
  python -c "import json;d=json.load(open('gpurun_out/wl_${tag}_$name.json'));r=d['roofline'];print('$name', d['config']['workload'], d['value'], d['ms_per_step'], r['frac'], r['segments_per_sample'], r.get('sphere_tests_per_segment_executed'), r.get('box_tests_per_segment', r.get('wall_tests_per_segment_executed')), r.get('frac_executed'))"; }
run simple --scene simple --width 400 --height 300 --spp 64 --steps 20 --warmup 3 &&
run box_c2 --scene box --width 1024 --height 768 --spp 256 --steps 10 --warmup 2 &&
run mirror_c3 --scene box_mirror --width 1920 --height 1080 --spp 1024 --steps 3 --warmup 1 &&
run box_c4frame --scene box --width 3840 --height 2160 --spp 4096 --steps 1 --warmup 1 &&
run synth_c5 --scene synthetic:10000 --width 1920 --height 1080 --spp 1024 --steps 2 --warmup 1
