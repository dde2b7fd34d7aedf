mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_fast_math.py -k "bvh or synthetic or Bvh or wide or C5" > gpurun_out/r04c_pytest.log 2>&1; rc=$?
tail -3 gpurun_out/r04c_pytest.log; [ $rc -eq 0 ] || { tail -40 gpurun_out/r04c_pytest.log; exit $rc; }
bash tools/gpu_ab.sh pf "main nopf" 3 "--workload c5 --steps 3 --warmup 1"
