#!/bin/bash
# GPU suite on the in-tree (working-tree) library, then the interleaved A/B of ab/*.so
OUT=gpurun_out/${1:-ab}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $OUT/gpu_tests.log 2>&1; rc=$?
echo tests_rc=$rc; tail -2 $OUT/gpu_tests.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $OUT/gpu_tests.log | head -20; exit 1; }
REPS=${REPS:-3} STEPS=${STEPS:-200} timeout -k 10 600 tools/ab_bench.sh
