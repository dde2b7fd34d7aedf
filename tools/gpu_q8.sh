set -o pipefail
mkdir -p gpurun_out
PTGPU_LIB=cpu-path-tracing_amd/build/libptgpu_q8.so timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_fast_math.py -k "bvh or synthetic or wide" > gpurun_out/q8_parity.log 2>&1 && tail -3 gpurun_out/q8_parity.log && bash tools/gpu_ab.sh q8 "main q8 tdx1 tdx2" 2 "--workload c5 --steps 3 --warmup 1"
