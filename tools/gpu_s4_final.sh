#!/bin/bash
# Session 4 close: the round-end sequence on HEAD -- GPU suite, smoke(), the driver's bench command
OUT=gpurun_out/s4_final
mkdir -p $OUT
export PP3_REPORT_DIR=$OUT
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1; rc=$?; echo tests_rc=$rc; tail -2 $OUT/gpu_tests.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || exit 1
tail -1 $OUT/smoke.log
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $OUT/bench_driver.json 2>&1 || exit 1
python3 -c "import json; d=json.loads(open('$OUT/bench_driver.json').read().strip().split('\n')[-1]); print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['state_sha16'], d['roofline'].get('fp32_vector', {}).get('frac'))"
