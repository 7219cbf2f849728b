#!/bin/bash
# Session 4: leg-leg Hessian accumulation restricted to the joined legs -- edge/physics tests on the
# in-tree build, then the interleaved A/B against HEAD at the driver's window and over 200 steps
OUT=gpurun_out/s4h
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_edge.py tests/test_gpu_physics.py -x -q --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?; echo tests_rc=$rc; tail -1 $OUT/tests.log
[ $rc -eq 0 ] || exit 1
REPS=4 STEPS=20 timeout -k 10 400 tools/ab_bench.sh > $OUT/ab20.txt 2>&1 || exit 1
cat $OUT/ab20.txt
REPS=2 STEPS=200 timeout -k 10 400 tools/ab_bench.sh > $OUT/ab200.txt 2>&1 || exit 1
cat $OUT/ab200.txt
