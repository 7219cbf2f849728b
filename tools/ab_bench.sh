#!/bin/bash
# A/B timing of kernel variants on the GPU box (via gpurun): each .so under ab/ is benched
# REPS times, interleaved (v1 v2 ... v1 v2 ...), on the driver's early-episode workload
# (configs[1], warmup 5) -> gpurun_out/ab/<tag>_<rep>.log; one summary line per run, with the end
# state's hash: variants with equal hashes ran the same trajectories (a pure code-speed comparison).
set -e
mkdir -p gpurun_out/ab
REPS=${REPS:-3}
STEPS=${STEPS:-200}
for rep in $(seq 1 $REPS); do
  for so in ab/*.so; do
    tag=$(basename $so .so)
    PP3_LIB_PATH=$PWD/$so timeout -k 10 120 python3 bench.py --steps $STEPS --warmup 5 --no-cpu-baseline --no-extras --no-latency-floor > gpurun_out/ab/${tag}_$rep.log 2>&1
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/ab/${tag}_$rep.log').read().strip().split('\n')[-1]); print('$tag', $rep, d['value'], d['roofline']['avg_launch_ms'], d.get('per_step_launch') and d['per_step_launch']['avg_launch_ms'], d.get('state_sha16'))"
  done
done
