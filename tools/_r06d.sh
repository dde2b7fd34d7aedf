set -o pipefail
bash tools/gpu_vmem_pmc.sh r06d_c5_packets --workload c5 > gpurun_out/r06d_vmem_c5_packets.txt 2>&1 || { echo pmc1 failed; tail gpurun_out/r06d_vmem_c5_packets.txt; exit 1; }
bash tools/gpu_vmem_pmc.sh r06d_c5_perlane --workload c5 --no-camera-packets > gpurun_out/r06d_vmem_c5_perlane.txt 2>&1 || { echo pmc2 failed; tail gpurun_out/r06d_vmem_c5_perlane.txt; exit 1; }
tail -12 gpurun_out/r06d_vmem_c5_packets.txt; tail -12 gpurun_out/r06d_vmem_c5_perlane.txt
