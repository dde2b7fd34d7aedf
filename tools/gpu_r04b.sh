mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_fast_math.py tests/test_gpu_reference.py tests/test_gpu_statistical.py > gpurun_out/r04b_pytest.log 2>&1; rc=$?
tail -15 gpurun_out/r04b_pytest.log | grep -v "^$"; grep -E "fast-vs-A/xs" gpurun_out/r04b_pytest.log | head; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_ab.sh nfr "main nfr" 2 "--steps 3 --warmup 1;--workload c3 --steps 2 --warmup 1;--workload c1 --steps 20 --warmup 3"
