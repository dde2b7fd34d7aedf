#!/usr/bin/env bash
# Round 5: the diffuse sampler without zero-initialised values for other
# lanes (noinit), and the split tail of small shards (tc16: 16 chunks per
# tail pixel group instead of 8; tl2: two tail levels, 8 then 16 chunks)
# measured with the single-GPU shard simulation of the bench frame.
tag=${1:-r05k}
mkdir -p gpurun_out
PTGPU_LIB=cpu-path-tracing_amd/build/libptgpu_noinit.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 \
  --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_fast_math.py -k "not cli" \
  > gpurun_out/${tag}_noinit_tests.log 2>&1 || { echo "noinit tests failed"; tail -15 gpurun_out/${tag}_noinit_tests.log; exit 1; }
echo "noinit: $(tail -1 gpurun_out/${tag}_noinit_tests.log)"
bash tools/gpu_ab.sh ${tag} "main noinit" 3 "--steps 3 --warmup 1;--workload c3 --steps 3 --warmup 1"
for v in tc16 tl2; do
  PTGPU_LIB=cpu-path-tracing_amd/build/libptgpu_$v.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 \
    --timeout-method thread -m gpu tests/test_gpu_parity.py -k "shard or tail or full" > gpurun_out/${tag}_${v}_tests.log 2>&1 \
    || { echo "$v tests failed"; tail -15 gpurun_out/${tag}_${v}_tests.log; exit 1; }
  echo "$v: $(tail -1 gpurun_out/${tag}_${v}_tests.log)"
done
for v in main tc16 tl2 main tc16 tl2; do
  lib=cpu-path-tracing_amd/build/libptgpu_$v.so; [ $v = main ] && lib=cpu-path-tracing_amd/libptgpu.so
  PTGPU_LIB=$lib timeout -k 10 300 python tools/shard_sim.py --counts 1 4 8 > gpurun_out/${tag}_ss_$v.json 2>/dev/null || { echo "$v shard_sim failed"; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/${tag}_ss_$v.json').read().strip().splitlines()[-1]);s=d['shards'];print('$v', {k:(round(v['max_ms'],3), v['efficiency_vs_first']) for k,v in s.items()})"
done
