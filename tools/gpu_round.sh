#!/bin/bash
# One GPU-box session (via gpurun): GPU parity suite, the driver's bench command, then the profile
# recipe (kernel-trace stats + separate PMC passes).  Every GPU step has its own time limit; a test
# FAILURE (pytest rc 1) still lets the bench run, anything worse (crash, abort, timeout) stops here.
#   tools/gpu_round.sh TAG [tests|notests]
TAG=${1:-r02}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export PP3_REPORT_DIR=$OUT
if [ "${2:-tests}" = tests ]; then
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread > $OUT/gpu_tests.log 2>&1
  rc=$?
  echo "tests_rc=$rc"; tail -n 25 $OUT/gpu_tests.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
fi
timeout -k 10 240 python3 bench.py --steps 20 --warmup 5 > $OUT/bench_driver.json 2> $OUT/bench_driver.err || { echo bench failed; tail -20 $OUT/bench_driver.err; exit 1; }
tail -c 3000 $OUT/bench_driver.json
bash tools/gpu_profile.sh $TAG/prof || { echo profile failed; exit 1; }
echo done
