#!/bin/bash
# The round-end sequence on the working tree (via gpurun): GPU parity suite, smoke(), the driver's
# bench command.  Every GPU step has its own time limit; the first failure ends the call.
#   tools/gpu_check.sh TAG [pytest -k expression]
TAG=${1:-check}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export PP3_REPORT_DIR=$OUT
K=${2:+-k "$2"}
eval timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread $K > $OUT/gpu_tests.log 2>&1
rc=$?; echo "tests_rc=$rc"; tail -n 4 $OUT/gpu_tests.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 240 python bench.py --steps 20 --warmup 5 > $OUT/bench_driver.json 2> $OUT/bench_driver.err || { tail $OUT/bench_driver.err; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/bench_driver.json').read().strip().split('\n')[-1]); print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d.get('per_step_launch') and d['per_step_launch']['avg_launch_ms'], d['state_sha16'], d['n_gpus'])"
