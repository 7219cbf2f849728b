#!/bin/bash
# Round-5 GPU session (via gpurun): GPU suite, smoke, the driver's bench command (ls_cap,
# idle_start), the A/B of ab/*.so, the host-API loop under a kernel + HIP trace, then the profile
# recipe of the working-tree kernel.  Each GPU step has its own limit; a crash / timeout ends it.
#   tools/gpu_r05.sh TAG [steps...]   steps: tests smoke driver ab abdrv hostapi parts prof phases policy
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export PP3_REPORT_DIR=$OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
rc=0
for step in "$@"; do
  case $step in
    tests)
      timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1
      rc=$?; echo "tests_rc=$rc"; grep -E "FAILED|ERROR" $OUT/gpu_tests.log | head -20; tail -n 2 $OUT/gpu_tests.log
      if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi ;;
    smoke)
      timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail $OUT/smoke.log; exit 1; }
      tail -2 $OUT/smoke.log ;;
    driver)
      timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $OUT/bench_driver.json 2> $OUT/bench_driver.err || { tail $OUT/bench_driver.err; exit 1; }
      python tools/bench_summary.py $OUT/bench_driver.json ;;
    ab)
      REPS=${REPS:-3} STEPS=${STEPS:-200} bash tools/ab_bench.sh > $OUT/ab.txt 2>&1 || { tail $OUT/ab.txt; exit 1; }
      cat $OUT/ab.txt ;;
    abdrv)
      REPS=${REPS:-4} STEPS=20 bash tools/ab_bench.sh > $OUT/ab_driver.txt 2>&1 || { tail $OUT/ab_driver.txt; exit 1; }
      cat $OUT/ab_driver.txt ;;
    hostapi)
      for mode in sync async_zc defer1 defer defer_read sync async_zc defer1 defer defer_read; do
        for pipe in 1 0; do
          timeout -k 10 200 python tools/host_api_trace.py 200 $pipe $mode >> $OUT/host_api_plain.txt 2>&1 || { tail $OUT/host_api_plain.txt; exit 1; }
        done
      done
      cat $OUT/host_api_plain.txt
      for mode in sync defer; do
        timeout -k 10 240 rocprofv3 --kernel-trace --hip-trace --stats -d $OUT/host_api_trace_$mode -o run --output-format csv -- python3 tools/host_api_trace.py 200 1 $mode > $OUT/host_api_trace_$mode.log 2>&1 || { tail $OUT/host_api_trace_$mode.log; exit 1; }
        grep "env.step" $OUT/host_api_trace_$mode.log
      done ;;
    prof)
      bash tools/gpu_profile.sh $TAG/prof > $OUT/prof.log 2>&1 || { tail -30 $OUT/prof.log; exit 1; }
      tail -30 $OUT/prof.log ;;
    phases)
      PP3_DIAG_OUT=$OUT DIAG_FUSED=1 timeout -k 10 300 python tests/diag_phases.py > $OUT/phases_fused.txt 2>&1 || { tail $OUT/phases_fused.txt; exit 1; }
      head -22 $OUT/phases_fused.txt
      python tools/trace_intervals.py $OUT/waves.npy 10,12,11,17,18,0 > $OUT/phases_fused_intervals.txt 2>&1; head -40 $OUT/phases_fused_intervals.txt ;;
    parts)
      timeout -k 10 300 python tools/host_api_parts.py 100 > $OUT/host_api_parts.txt 2>&1 || { tail $OUT/host_api_parts.txt; exit 1; }
      cat $OUT/host_api_parts.txt ;;
    policy)
      timeout -k 10 300 python bench.py --policy 256,128,128 > $OUT/bench_policy.json 2> $OUT/bench_policy.err || { tail $OUT/bench_policy.err; exit 1; }
      python tools/bench_summary.py $OUT/bench_policy.json
      timeout -k 10 300 python bench.py --policy 256,128,128 --steps 20 --warmup 5 > $OUT/bench_policy_drv.json 2> $OUT/bench_policy_drv.err || { tail $OUT/bench_policy_drv.err; exit 1; }
      python tools/bench_summary.py $OUT/bench_policy_drv.json ;;
  esac
done
exit $rc
