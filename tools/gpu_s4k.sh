#!/bin/bash
# Session 4: policy MLP with / without the L2 weight prefetch at kernel start, layer-shape sweep;
# then the policy parity test on the prefetch build
OUT=gpurun_out/s4k
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
for v in nopf pf nopf2 pf2; do
  so=ab/${v%2}.so
  PP3_LIB_PATH=$PWD/$so timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $OUT/$v -o run -- python3 tools/policy_sweep.py > $OUT/$v.log 2>&1 || exit 1
  echo "== $v"; python3 tools/policy_sweep_summary.py $OUT/$v
done
PP3_LIB_PATH=$PWD/ab/pf.so timeout -k 10 200 python -u -m pytest tests/test_gpu_policy.py -x -q --timeout 150 --timeout-method thread > $OUT/policy_tests.log 2>&1; echo policy_tests_rc=$?; tail -1 $OUT/policy_tests.log
