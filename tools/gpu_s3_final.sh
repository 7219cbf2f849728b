#!/bin/bash
# session-3 close: GPU suite, driver bench, profile recipe (kernel trace + PMC passes)
OUT=gpurun_out/s3f
mkdir -p $OUT
export PP3_REPORT_DIR=$OUT
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $OUT/gpu_tests.log 2>&1; rc=$?; echo tests_rc=$rc; tail -3 $OUT/gpu_tests.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $OUT/bench_driver.json 2>&1 || exit 1
tail -c 400 $OUT/bench_driver.json
tools/gpu_profile.sh s3prof || exit 1
