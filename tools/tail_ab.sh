set -e
for v in main h3 main h3; do
  lib=cpu-path-tracing_amd/build/libptgpu_$v.so; [ $v = main ] && lib=cpu-path-tracing_amd/libptgpu.so
  PTGPU_LIB=$lib timeout -k 10 200 python tools/shard_sim.py --counts 1 2 4 8 --steps 3 > gpurun_out/ss_$v.json 2> gpurun_out/ss_$v.err
  echo "$v $(cat gpurun_out/ss_$v.json)"
done
