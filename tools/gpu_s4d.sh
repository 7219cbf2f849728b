#!/bin/bash
# Session 4: configs[3] per GPU with the per-step RCCL hand-over (one-rank communicator on one GPU),
# gather to a root and all-gather
OUT=gpurun_out/s4d
mkdir -p $OUT
timeout -k 10 300 python3 bench.py --envs 8192 --random-commands --gather --no-cpu-baseline > $OUT/bench_c4_gather.log 2>&1 || exit 1
tail -n 1 $OUT/bench_c4_gather.log > $OUT/bench_c4_gather.json
timeout -k 10 300 python3 bench.py --envs 8192 --random-commands --gather --gather-root -1 --no-cpu-baseline --no-extras > $OUT/bench_c4_allgather.log 2>&1 || exit 1
tail -n 1 $OUT/bench_c4_allgather.log > $OUT/bench_c4_allgather.json
for f in $OUT/bench_c4_gather.json $OUT/bench_c4_allgather.json; do python3 -c "import json; d=json.load(open('$f')); print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], json.dumps(d['config']['gather']), d['config']['comm'])"; done
