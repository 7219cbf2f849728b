#!/bin/bash
# PC sampling (stochastic, stall reasons) of the bench's env_step_kernel -> gpurun_out/$TAG/pcs
TAG=${1:-pcs}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -s KILL 120 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method stochastic --pc-sampling-unit cycles \
  --pc-sampling-interval ${2:-65536} -d $OUT/pcs -o run --output-format csv -- \
  python3 bench.py --steps 200 --warmup 5 --no-cpu-baseline --no-latency-floor --no-extras > $OUT/pcs.log 2>&1
