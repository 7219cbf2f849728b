#!/bin/bash
# Quick GPU iteration (via gpurun): GPU parity tests, bench line, phase breakdown -> gpurun_out/$1/
set -e
OUT=gpurun_out/${1:-quick}
mkdir -p $OUT
timeout -k 10 400 python3 -m pytest tests -m gpu -x -q > $OUT/gpu_tests.log 2>&1
timeout -k 10 240 python3 bench.py --no-cpu-baseline > $OUT/bench.log 2>&1
timeout -k 10 240 python3 tests/diag_phases.py > $OUT/phases.log 2>&1
