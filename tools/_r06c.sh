set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_fast_math.py tests/test_gpu_parity.py > gpurun_out/r06c_tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/r06c_tests.log; exit 1; }
tail -1 gpurun_out/r06c_tests.log
bash tools/gpu_ab.sh r06c "main main:--no-camera-packets" 3 "--workload c5 --steps 3 --warmup 1"
bash tools/gpu_ab.sh r06c "main main:--generic-scan" 3 "--steps 3 --warmup 1;--workload c3 --steps 3 --warmup 1"
