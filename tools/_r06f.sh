set -o pipefail
mkdir -p gpurun_out
PTGPU_LIB=cpu-path-tracing_amd/build/libptgpu_coop.so timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_fast_math.py -k "bvh or synthetic or wide" > gpurun_out/r06f_coop_tests.log 2>&1 || { echo coop tests failed; tail -20 gpurun_out/r06f_coop_tests.log; exit 1; }
tail -1 gpurun_out/r06f_coop_tests.log
bash tools/gpu_ab.sh r06f "main coop" 3 "--workload c5 --steps 3 --warmup 1"
PTGPU_LIB=cpu-path-tracing_amd/build/libptgpu_coop.so bash tools/gpu_vmem_pmc.sh r06f_c5_coop --workload c5 > gpurun_out/r06f_vmem_c5_coop.txt 2>&1 || { echo pmc failed; tail gpurun_out/r06f_vmem_c5_coop.txt; exit 1; }
tail -9 gpurun_out/r06f_vmem_c5_coop.txt
