#!/bin/bash
# Session 4: the comm tests incl. the configs[3]-size gather
OUT=gpurun_out/s4g
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_comm.py -x -v --timeout 200 --timeout-method thread > $OUT/comm_tests.log 2>&1; rc=$?; echo rc=$rc; grep -E "PASS|FAIL|Error|assert" $OUT/comm_tests.log | tail -12
exit $rc
