#!/bin/bash
# Profile recipe run on the GPU box (via gpurun) -- writes under gpurun_out/$TAG/.
#   kernel-trace stats pass, then separate PMC passes (SQ instruction mix, FETCH_SIZE, WRITE_SIZE),
#   each under its own time limit; stops at the first failure.
set -e
TAG=${1:-prof}
ARGS=${2:---steps 50 --warmup 5 --no-cpu-baseline --no-latency-floor --no-extras}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py $ARGS > $OUT/trace.log 2>&1
timeout -k 10 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY -d $OUT/pmc_sq -o run --output-format csv -- python3 bench.py $ARGS > $OUT/pmc_sq.log 2>&1
timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o run --output-format csv -- python3 bench.py $ARGS > $OUT/pmc_fetch.log 2>&1
timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o run --output-format csv -- python3 bench.py $ARGS > $OUT/pmc_write.log 2>&1
python3 tools/summarize_profile.py $OUT
