#!/bin/bash
# GPU suite on the in-tree (working-tree) library, then interleaved A/B of ab/*.so at the driver's
# window (20 steps) and over 200 steps.   tools/gpu_ab2.sh TAG [tests|notests]
OUT=gpurun_out/${1:-ab}
mkdir -p $OUT
export PP3_REPORT_DIR=$OUT
if [ "${2:-tests}" = tests ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1; rc=$?
  echo tests_rc=$rc; tail -2 $OUT/gpu_tests.log
  [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $OUT/gpu_tests.log | head -20; exit 1; }
fi
REPS=${REPS20:-4} STEPS=20 timeout -k 10 600 tools/ab_bench.sh || exit 1
REPS=${REPS200:-2} STEPS=200 timeout -k 10 600 tools/ab_bench.sh
