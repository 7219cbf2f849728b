#!/bin/bash
# Scalar-cache PMC passes for env_step_kernel (model constants are read with s_load; the scalar
# and LDS loads share lgkmcnt, so a scalar miss also lengthens the LDS waits behind it).
# One rocprofv3 --pmc run per pass, each under its own time limit; stops at the first failure.
TAG=${1:-sqc}
ARGS=${2:---steps 50 --warmup 5 --no-cpu-baseline --no-latency-floor --no-extras}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
run() {  # name counters...
  local name=$1; shift
  timeout -s KILL 90 rocprofv3 --pmc "$@" -d $OUT/$name -o run --output-format csv -- python3 bench.py $ARGS > $OUT/$name.log 2>&1 || { echo "pass $name failed"; tail -5 $OUT/$name.log; exit 1; }
}
run dcache SQ_WAVES SQC_DCACHE_REQ SQC_DCACHE_HITS SQC_DCACHE_MISSES SQC_DCACHE_MISSES_DUPLICATE SQ_INSTS_SMEM
run icache SQ_WAVES SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_WAVE_CYCLES
run smemlat SmemLatency
run ldslat LdsLatency
echo all passes ok
