#!/usr/bin/env bash
# Single-GPU-box rehearsal of the N-rank bench path: N ranks share cuda:0 and
# gather over gloo (PTG_REHEARSAL=1).  The real N-GPU run uses RCCL.
n=${1:-2}; shift || true
PTG_REHEARSAL=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus $n --steps 2 --warmup 1 "$@" \
  > gpurun_out/rehearse_$n.json 2> gpurun_out/rehearse_$n.err
rc=$?; echo "rehearsal n=$n rc=$rc"; cut -c1-600 gpurun_out/rehearse_$n.json; exit $rc
