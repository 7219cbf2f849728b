#!/bin/bash
# Session-4 check of a fresh-container build: GPU suite, then the driver's bench command
OUT=gpurun_out/s4
mkdir -p $OUT
export PP3_REPORT_DIR=$OUT
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $OUT/gpu_tests.log 2>&1; rc=$?; echo tests_rc=$rc; tail -2 $OUT/gpu_tests.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $OUT/bench_driver.json 2>&1 || exit 1
tail -c 400 $OUT/bench_driver.json
