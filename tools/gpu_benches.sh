#!/bin/bash
# All bench configurations, one JSON line each -> gpurun_out/$1/bench_<cfg>.json
set -e
OUT=gpurun_out/${1:-benches}
mkdir -p $OUT
run() { local name=$1; shift; timeout -k 10 300 python3 bench.py "$@" > $OUT/bench_$name.log 2>&1; tail -n 1 $OUT/bench_$name.log > $OUT/bench_$name.json; echo "$name $(python3 -c "import json; d=json.load(open('$OUT/bench_$name.json')); p=d.get('per_step_launch') or {}; print(d['value'], d['roofline']['avg_launch_ms'], p.get('avg_launch_ms'), p.get('bit_equal_to_rollout'))")"; }
run driver --steps 20 --warmup 5
run driver_step --steps 20 --warmup 5 --launch step --no-cpu-baseline
run default
run dr --dr --no-cpu-baseline
run obst --obstacles 10 --no-cpu-baseline
run terrain --obstacles 10 --terrain --no-cpu-baseline
run autoreset --auto-reset 1000 --no-cpu-baseline
run policy --policy 256,128,128 --no-cpu-baseline
run envs8192 --envs 8192 --no-cpu-baseline
run c4 --envs 8192 --random-commands --no-cpu-baseline
run c4_gather --envs 8192 --random-commands --gather --no-cpu-baseline
run policy_drv --policy 256,128,128 --steps 20 --warmup 5 --no-cpu-baseline
run policy8192 --policy 256,128,128 --envs 8192 --no-cpu-baseline
run policy8192_drv --policy 256,128,128 --envs 8192 --steps 20 --warmup 5 --no-cpu-baseline
run c4_unroll_gather --envs 8192 --random-commands --gather --gather-mode unroll --no-cpu-baseline
