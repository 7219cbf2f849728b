#!/bin/bash
# A focused GPU-box session (via gpurun): the named GPU test files, smoke(), the driver's bench
# command, then any extra bench flag sets given in $BENCH_EXTRA (';'-separated).  Every GPU step
# has its own time limit; the first crash / timeout ends the call, a test FAILURE (pytest rc 1)
# still lets smoke and the bench run.
#   [BENCH_EXTRA="--policy 256,128,128;--dr"] tools/gpu_quick.sh TAG test_file...
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export PP3_REPORT_DIR=$OUT
rc=0
if [ $# -gt 0 ]; then
  timeout -k 10 900 python -u -m pytest "$@" -m gpu -v --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1
  rc=$?; echo "tests_rc=$rc"; grep -E "PASSED|FAILED|ERROR" $OUT/gpu_tests.log | tail -n 60; tail -n 3 $OUT/gpu_tests.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
fi
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
summ() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().split('\n')[-1]); r=d['roofline']; print(sys.argv[1], d['value'], d['ms_per_step'], r['avg_launch_ms'], d.get('per_step_launch') and d['per_step_launch'].get('avg_launch_ms'), d.get('state_sha16'), r.get('binding'), d.get('cpu_baseline', {}).get('cores'), d.get('cpu_baseline', {}).get('host_cores'))" $1; }
timeout -k 10 240 python bench.py --steps 20 --warmup 5 > $OUT/bench_driver.json 2> $OUT/bench_driver.err || { tail $OUT/bench_driver.err; exit 1; }
summ $OUT/bench_driver.json
i=0
IFS=';' read -ra EXTRA <<< "${BENCH_EXTRA:-}"
for flags in "${EXTRA[@]}"; do
  i=$((i+1))
  timeout -k 10 240 python bench.py $flags > $OUT/bench_extra_$i.json 2> $OUT/bench_extra_$i.err || { tail $OUT/bench_extra_$i.err; exit 1; }
  echo "extra $i: $flags"; summ $OUT/bench_extra_$i.json
done
exit $rc
