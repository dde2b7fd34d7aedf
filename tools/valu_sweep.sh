#!/usr/bin/env bash
# Dynamic instruction counts + time per library variant (build/libptgpu_<name>.so;
# "main" = the in-tree libptgpu.so).  Usage: bash tools/valu_sweep.sh "<names>" [bench args...]
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
names=$1; shift || true
for n in $names; do
  lib=cpu-path-tracing_amd/build/libptgpu_$n.so; [ "$n" = main ] && lib=cpu-path-tracing_amd/libptgpu.so
  d=gpurun_out/vs_$n; rm -rf $d; mkdir -p $d
  PTGPU_LIB=$lib timeout -k 10 120 python bench.py --steps 3 --warmup 1 --cpu-baseline off "$@" > $d/bench.json 2>/dev/null || { echo "$n bench failed"; exit 1; }
  PTGPU_LIB=$lib timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES GRBM_GUI_ACTIVE -d $d/pmc -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --cpu-baseline off "$@" > $d/bench_pmc.json 2> $d/pmc.err || { echo "$n pmc failed"; exit 1; }
  python3 - "$d" "$n" <<'PY'
import csv, json, sys, collections
d, n = sys.argv[1], sys.argv[2]
b = json.load(open(f"{d}/bench.json"))
agg = collections.defaultdict(list)
for r in csv.DictReader(open(f"{d}/pmc/run_counter_collection.csv")):
    if "render_kernel" in r["Kernel_Name"]:
        agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
c = {k: sum(v) / len(v) for k, v in agg.items()}
samples = b["config"]["width"] * b["config"]["height"] * b["config"]["spp"]
wseg = b["roofline"]["segments_per_sample"] * samples / 64
cyc = c["GRBM_GUI_ACTIVE"] / 8
print(f"{n}: {b['ms_per_step']:.2f} ms  {b['value']:.0f} Ms/s  VALU/seg {c['SQ_INSTS_VALU']/wseg:.1f}  SALU/seg {c['SQ_INSTS_SALU']/wseg:.1f}  LDS/seg {c['SQ_INSTS_LDS']/wseg:.2f}  valu_issue {100*c['SQ_INSTS_VALU']*2/1024/cyc:.1f}%")
PY
done
