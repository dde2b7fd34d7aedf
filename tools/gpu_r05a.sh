#!/usr/bin/env bash
# Round 5, first GPU pass on HEAD: the -m gpu suite, the default bench line
# (N = 1, CPU baseline included), and the two 1-GPU rehearsals of the N > 1
# paths on the metric's frame (in-process ptg_multi with 4 local shards;
# torchrun with 2 gloo ranks) -- their lines must name the same workload.
# Usage (GPU box): bash tools/gpu_r05a.sh <tag>
tag=${1:-r05a}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/${tag}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/${tag}_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err \
  || { echo BENCH FAILED; tail gpurun_out/${tag}_bench.err; exit 1; }
cut -c1-400 gpurun_out/${tag}_bench.json
PTG_REHEARSAL=1 timeout -k 10 300 python bench.py --gpus 4 --steps 2 --warmup 1 --t1-steps 1 \
  > gpurun_out/${tag}_rehearse4_inprocess.json 2> gpurun_out/${tag}_rehearse4_inprocess.err \
  || { echo REHEARSAL4 FAILED; tail gpurun_out/${tag}_rehearse4_inprocess.err; exit 1; }
cut -c1-300 gpurun_out/${tag}_rehearse4_inprocess.json
PTG_REHEARSAL=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 2 --warmup 1 --t1-steps 1 \
  > gpurun_out/${tag}_rehearse2_torchrun.json 2> gpurun_out/${tag}_rehearse2_torchrun.err \
  || { echo REHEARSAL2 FAILED; tail gpurun_out/${tag}_rehearse2_torchrun.err; exit 1; }
cut -c1-300 gpurun_out/${tag}_rehearse2_torchrun.json
echo done
