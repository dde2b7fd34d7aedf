#!/usr/bin/env bash
# HBM write bytes (rocprofv3 --pmc WRITE_SIZE) of the C5 render kernel per
# library variant, next to its frame time.  Usage: bash tools/bvh_write_ab.sh "<variants>"
set -e
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
C5="--scene synthetic:10000 --width 1920 --height 1080 --spp 1024 --steps 1 --warmup 1 --cpu-baseline off"
for v in $1; do
  lib=cpu-path-tracing_amd/build/libptgpu_$v.so; [ $v = main ] && lib=cpu-path-tracing_amd/libptgpu.so
  out=gpurun_out/wr_$v; mkdir -p $out
  PTGPU_LIB=$lib timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE -d $out -o run --output-format csv -- python3 bench.py $C5 > $out/bench.json 2> $out/err
  python - "$out" "$v" <<'PY'
import csv, glob, json, sys
out, v = sys.argv[1], sys.argv[2]
rows = [r for f in glob.glob(out + "/**/run_counter_collection.csv", recursive=True) for r in csv.DictReader(open(f))]
w = [float(r["Counter_Value"]) for r in rows if "render_kernel" in r["Kernel_Name"]]
sc = {r["Scratch_Size"] for r in rows if "render_kernel" in r["Kernel_Name"]}
d = json.loads(open(out + "/bench.json").read().strip().splitlines()[-1])
print(v, "ms", d["ms_per_step"], "render WRITE_SIZE MB per launch", round(sum(w) / len(w) * 1024 / 1e6, 1), "scratch", sc)
PY
done
