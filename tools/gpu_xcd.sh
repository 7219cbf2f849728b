#!/bin/bash
# XCD-aware mapping check: GPU suite, A/B vs HEAD, FETCH/WRITE_SIZE passes of the working tree
OUT=gpurun_out/xcd
mkdir -p $OUT
tools/gpu_ab.sh xcd || exit 1
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
ARGS="--steps 50 --warmup 5 --no-cpu-baseline --no-latency-floor --no-extras"
timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o run --output-format csv -- python3 bench.py $ARGS > $OUT/pmc_fetch.log 2>&1 || exit 1
timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o run --output-format csv -- python3 bench.py $ARGS > $OUT/pmc_write.log 2>&1 || exit 1
find $OUT -name "*counter_collection*" | head
