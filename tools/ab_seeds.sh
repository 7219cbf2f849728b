#!/bin/bash
# A/B over several bench seeds (different trajectories): for edits that change rounding, the
# per-trajectory work differences average out across seeds.  ab/*.so interleaved per seed.
mkdir -p gpurun_out/abs
SEEDS=${SEEDS:-"1 2 3 4 5"}
STEPS=${STEPS:-200}
for seed in $SEEDS; do
  for so in ab/*.so; do
    tag=$(basename $so .so)
    PP3_LIB_PATH=$PWD/$so timeout -k 10 120 python3 bench.py --seed $seed --steps $STEPS --warmup 5 --no-cpu-baseline --no-extras --no-latency-floor > gpurun_out/abs/${tag}_$seed.log 2>&1 || exit 1
    python3 -c "import json; d=json.loads(open('gpurun_out/abs/${tag}_$seed.log').read().strip().split('\n')[-1]); print('$tag', $seed, d['value'], d['roofline']['avg_launch_ms'], d.get('per_step_launch') and d['per_step_launch']['avg_launch_ms'], d.get('state_sha16'))"
  done
done
