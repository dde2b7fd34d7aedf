#!/usr/bin/env bash
# Round-end style check on HEAD (GPU box), as the driver runs it: the -m gpu
# suite, __graft_entry__.smoke(), the default bench line (N = 1, CPU
# baseline included) and the two 1-GPU rehearsals of the N > 1 paths.
# Usage: bash tools/gpu_check.sh <tag>
tag=${1:-final}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/${tag}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/${tag}_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${tag}_smoke.log 2>&1 \
  || { echo SMOKE FAILED; tail -20 gpurun_out/${tag}_smoke.log; exit 1; }
tail -1 gpurun_out/${tag}_smoke.log
timeout -k 10 300 python bench.py > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err \
  || { echo BENCH FAILED; tail gpurun_out/${tag}_bench.err; exit 1; }
cut -c1-400 gpurun_out/${tag}_bench.json
PTG_REHEARSAL=1 timeout -k 10 300 python bench.py --gpus 8 --steps 2 --warmup 1 --t1-steps 1 \
  > gpurun_out/${tag}_rehearse8_inprocess.json 2> gpurun_out/${tag}_rehearse8_inprocess.err \
  || { echo REHEARSAL8 FAILED; tail gpurun_out/${tag}_rehearse8_inprocess.err; exit 1; }
cut -c1-300 gpurun_out/${tag}_rehearse8_inprocess.json
echo done
