#!/bin/bash
# Interleaved A/B of the ab/*.so variants over several bench workloads (via gpurun): for each rep,
# each workload, each variant one bench.py run -> one summary line (value, launch ms, end-state
# hash); ab/<tag>.env, if present, holds extra KEY=VALUE environment for ab/<tag>.so.
#   AB_SETS="--steps 20 --warmup 5;--obstacles 10;--obstacles 10 --terrain" REPS=2 tools/ab_flags_bench.sh
set -e
mkdir -p gpurun_out/ab
REPS=${REPS:-2}
IFS=';' read -ra SETS <<< "${AB_SETS:---steps 20 --warmup 5}"
for rep in $(seq 1 $REPS); do
  i=0
  for flags in "${SETS[@]}"; do
    i=$((i+1))
    for so in ab/*.so; do
      tag=$(basename $so .so)
      log=gpurun_out/ab/${tag}_s${i}_$rep.log
      envf=ab/$tag.env  # optional KEY=VALUE lines for this variant (e.g. PP3_NO_CULL=1)
      env PP3_LIB_PATH=$PWD/$so $( [ -f $envf ] && cat $envf ) timeout -k 10 150 python3 bench.py $flags --no-cpu-baseline --no-extras --no-latency-floor > $log 2>&1
      python3 -c "import json,sys; d=json.loads(open('$log').read().strip().split('\n')[-1]); print('$tag', 'set$i', $rep, d['value'], d['roofline']['avg_launch_ms'], d.get('per_step_launch') and d['per_step_launch']['avg_launch_ms'], d.get('state_sha16'))"
    done
  done
done
