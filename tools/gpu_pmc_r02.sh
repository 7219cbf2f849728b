#!/bin/bash
# Stall-attribution PMC passes for env_step_kernel (one rocprofv3 --pmc run per group, each
# under its own time limit; stops at the first failure).  Output: gpurun_out/$TAG/<pass>/
TAG=${1:-pmc2}
ARGS=${2:---steps 50 --warmup 5 --no-cpu-baseline --no-latency-floor --no-extras}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
run() {  # name counters...
  local name=$1; shift
  timeout -s KILL 90 rocprofv3 --pmc "$@" -d $OUT/$name -o run --output-format csv -- python3 bench.py $ARGS > $OUT/$name.log 2>&1 || { echo "pass $name failed"; exit 1; }
}
run active SQ_WAVES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_VMEM SQ_INSTS_BRANCH
run mix SQ_WAVES SQ_INSTS_SMEM SQ_INST_CYCLES_SALU SQ_INSTS_VALU_TRANS_F32 SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_LDS
run waits SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_IFETCH
run ldslat LdsLatency
run smemlat SmemLatency
run vmemlat VmemLatency
run ifetch InstrFetchLatency
echo all passes ok
