mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_multi.py tests/test_gpu_statistical.py tests/test_gpu_parity.py -k "multi or statistical or bvh or synthetic or Bvh or wide" > gpurun_out/r04a_pytest.log 2>&1 || { echo PYTEST FAILED; tail -30 gpurun_out/r04a_pytest.log; exit 1; }
tail -3 gpurun_out/r04a_pytest.log
timeout -k 10 200 python bench.py > gpurun_out/r04a_bench.json 2> gpurun_out/r04a_bench.err || { echo BENCH FAILED; tail gpurun_out/r04a_bench.err; exit 1; }
cut -c1-400 gpurun_out/r04a_bench.json
PTG_REHEARSAL=1 timeout -k 10 200 python bench.py --gpus 4 --steps 3 --warmup 1 > gpurun_out/r04a_rehearse4.json 2> gpurun_out/r04a_rehearse4.err || { echo REHEARSAL FAILED; tail gpurun_out/r04a_rehearse4.err; exit 1; }
cut -c1-300 gpurun_out/r04a_rehearse4.json
for r in 1 2; do for v in main nopos; do
  lib=cpu-path-tracing_amd/build/libptgpu_$v.so; [ $v = main ] && lib=cpu-path-tracing_amd/libptgpu.so
  PTGPU_LIB=$lib timeout -k 10 120 python bench.py --workload c5 --steps 3 --warmup 1 --cpu-baseline off > gpurun_out/r04a_c5_$v.json 2>/dev/null || { echo "c5 $v failed"; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r04a_c5_$v.json'));print('c5 $v', d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'])"
done; done
