#!/bin/bash
# Instruction/scalar-cache PMC pass for each ab/*.so (run on the GPU box via gpurun):
#   gpurun_out/icache/<tag>/ ; one rocprofv3 --pmc run per library, each under its own limit.
set -e
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
mkdir -p gpurun_out/icache
for so in ab/*.so; do
  tag=$(basename $so .so)
  PP3_LIB_PATH=$PWD/$so timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE -d gpurun_out/icache/$tag -o run --output-format csv -- python3 bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-latency-floor --no-extras > gpurun_out/icache/$tag.log 2>&1
done
echo icache passes ok
