#!/bin/bash
# Extra SQ counter passes (stall breakdown) for env_step_kernel -> gpurun_out/$1/
set -e
OUT=gpurun_out/${1:-pmcd}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
ARGS="--steps 30 --warmup 5 --no-cpu-baseline --no-latency-floor"
timeout -k 10 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA -d $OUT/p1 -o run --output-format csv -- python3 bench.py $ARGS > $OUT/p1.log 2>&1
timeout -k 10 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_LDS_BANK_CONFLICT SQ_INST_CYCLES_VMEM_RD SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU -d $OUT/p2 -o run --output-format csv -- python3 bench.py $ARGS > $OUT/p2.log 2>&1
