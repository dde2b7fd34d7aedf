#!/usr/bin/env bash
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r06an
timeout -s KILL 200 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES -d gpurun_out/r06an/lds -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --cpu-baseline off > gpurun_out/r06an/bench.json 2> gpurun_out/r06an/lds.err
echo rc=$?
