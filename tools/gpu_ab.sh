#!/usr/bin/env bash
# Same-box A/B of library variants on bench workloads (interleaved rounds).
# Usage (GPU box): bash tools/gpu_ab.sh <tag> "<variants>" <rounds> "<workload args>;<workload args>;..."
# variant "main" = cpu-path-tracing_amd/libptgpu.so, else build/libptgpu_<v>.so;
# "<v>:<bench args>" adds bench.py arguments (commas for spaces), e.g.
# "main main:--generic-scan"
tag=$1; vars=$2; rounds=$3; wls=$4
mkdir -p gpurun_out
IFS=';' read -ra W <<< "$wls"
for r in $(seq 1 $rounds); do
  for w in "${W[@]}"; do
    for tok in $vars; do
      v=${tok%%:*}; extra=""; [ "$tok" != "$v" ] && extra=${tok#*:} && extra=${extra//,/ }
      lib=cpu-path-tracing_amd/build/libptgpu_$v.so; [ $v = main ] && lib=cpu-path-tracing_amd/libptgpu.so
      name=$(echo "$tok" | tr -c 'A-Za-z0-9_\n' '_')
      out=gpurun_out/ab_${tag}_$name.json
      PTGPU_LIB=$lib timeout -k 10 150 python bench.py --cpu-baseline off $w $extra > $out 2>/dev/null || { echo "$tok [$w] failed"; exit 1; }
      python -c "import json;d=json.load(open('$out'));r=d['roofline'];print('$tok', d['config']['workload'], 'round $r', d['ms_per_step'], r['kernel_ms'], r['frac'], 'box/seg', r.get('box_tests_per_segment', r.get('wall_tests_per_segment_executed')), 'sph/seg', r.get('sphere_tests_per_segment_executed'), r.get('scan_kernel'))"
    done
  done
done
