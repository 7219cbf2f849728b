#!/bin/bash
# FP32 instruction-mix PMC pass (via gpurun): executed FP32 VALU operations of env_step_kernel
#   -> gpurun_out/$TAG/pmc_flops ; summarise with tools/summarize_flops.py gpurun_out/$TAG
set -e
TAG=${1:-flops}
ARGS=${2:---steps 50 --warmup 5 --no-cpu-baseline --no-latency-floor --no-extras}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_TRANS_F32 -d $OUT/pmc_flops -o run --output-format csv -- python3 bench.py $ARGS > $OUT/pmc_flops.log 2>&1
python3 tools/summarize_flops.py $OUT
