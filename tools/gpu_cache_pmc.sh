#!/usr/bin/env bash
# L1 (TCP) and L2 (TCC) hit counters of one workload's render kernel, one
# rocprofv3 --pmc pass per counter group.  Usage (GPU box):
#   bash tools/gpu_cache_pmc.sh <tag> [bench args]
tag=${1:-cache}; shift || true
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
out=gpurun_out/pmc_$tag; mkdir -p $out
B=(bench.py --steps 1 --warmup 1 --cpu-baseline off "$@")
timeout -s KILL 120 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum -d $out/tcp -o run --output-format csv -- python3 "${B[@]}" > $out/tcp.json 2> $out/tcp.err || { echo tcp failed; tail -3 $out/tcp.err; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d $out/tcc -o run --output-format csv -- python3 "${B[@]}" > $out/tcc.json 2> $out/tcc.err || { echo tcc failed; tail -3 $out/tcc.err; exit 1; }
python3 - "$out" <<'PY'
import csv, sys, collections
out = sys.argv[1]
v = collections.defaultdict(dict)
for sub in ("tcp", "tcc"):
    rows = list(csv.DictReader(open(f"{out}/{sub}/run_counter_collection.csv")))
    last = {}
    for r in rows:
        if "render_kernel<false" not in r["Kernel_Name"]:
            continue
        k = (r["Counter_Name"])
        d = int(r["Dispatch_Id"])
        if k not in last or d > last[k][0]:
            last[k] = (d, float(r["Counter_Value"]))
    for k, (d, x) in last.items():
        v["c"][k] = x
c = v["c"]
print(c)
if c.get("TCP_TOTAL_CACHE_ACCESSES_sum"):
    print("L1 miss fraction (TCP->TCC read requests / TCP accesses):", c["TCP_TCC_READ_REQ_sum"] / c["TCP_TOTAL_CACHE_ACCESSES_sum"])
if c.get("TCC_HIT_sum") is not None:
    print("L2 hit rate:", c["TCC_HIT_sum"] / (c["TCC_HIT_sum"] + c["TCC_MISS_sum"]))
PY
