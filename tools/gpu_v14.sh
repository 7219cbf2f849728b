#!/bin/bash
# v14 close: GPU suite, profile recipe, driver bench (after the profile so it reads the new traffic file), all configurations
OUT=gpurun_out/v14
mkdir -p $OUT
export PP3_REPORT_DIR=$OUT
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $OUT/gpu_tests.log 2>&1; rc=$?; echo tests_rc=$rc; tail -2 $OUT/gpu_tests.log
[ $rc -eq 0 ] || exit 1
tools/gpu_profile.sh v14prof || exit 1
python3 tools/summarize_profile.py gpurun_out/v14prof --commit gpurun_out/v14/r02_v14 > /dev/null || exit 1
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $OUT/bench_driver.json 2>&1 || exit 1
tail -c 300 $OUT/bench_driver.json
tools/gpu_benches.sh v14b || exit 1
PP3_LIB_PATH=$PWD/pupperv3-mjx_amd/pupperv3_mjx/libpupper_hip_prof.so PP3_DIAG_OUT=$OUT timeout -k 10 200 python tests/diag_phases.py > $OUT/phases.log 2>&1 || exit 1
head -3 $OUT/phases.log
