#!/bin/bash
# Session 4: the DR / terrain / auto-reset bench lines with per-env-model accuracy checks
OUT=gpurun_out/s4b
mkdir -p $OUT
run() { local name=$1; shift; timeout -k 10 300 python3 bench.py "$@" > $OUT/bench_$name.log 2>&1 || return 1; tail -n 1 $OUT/bench_$name.log > $OUT/bench_$name.json; python3 -c "import json; d=json.load(open('$OUT/bench_$name.json')); print('$name', d['value'], json.dumps(d['one_step_err']), d['qpos_rel_err']['value'])"; }
run dr --dr --no-cpu-baseline && run terrain --obstacles 10 --terrain --no-cpu-baseline && run autoreset --auto-reset 1000 --no-cpu-baseline
