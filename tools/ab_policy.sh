#!/bin/bash
# A/B of the policy-in-the-loop rollout (bench.py --policy) over the kernel variants under ab/:
# each .so REPS times, interleaved, on the driver's window (20 steps after 5 warmup steps) ->
# gpurun_out/ab_policy/<tag>_<rep>.log; one summary line per run (fused ms/step, the unfused
# replay's ms/step, actions / end state bit-equal, end-state hash).
mkdir -p gpurun_out/ab_policy
REPS=${REPS:-2}
STEPS=${STEPS:-20}
POLICY=${POLICY:-256,128,128}
for rep in $(seq 1 $REPS); do
  for so in ab/*.so; do
    tag=$(basename $so .so)
    PP3_LIB_PATH=$PWD/$so timeout -k 10 180 python3 bench.py --policy $POLICY --steps $STEPS --warmup 5 --no-cpu-baseline --no-extras > gpurun_out/ab_policy/${tag}_$rep.log 2>&1
    rc=$?
    if [ $rc -ne 0 ]; then echo "$tag $rep bench rc=$rc"; tail -3 gpurun_out/ab_policy/${tag}_$rep.log; [ $rc -ge 124 ] && exit $rc; continue; fi
    python3 -c "import json; d=json.loads(open('gpurun_out/ab_policy/${tag}_$rep.log').read().strip().split('\n')[-1]); p=d['per_step_launch']; print('$tag', $rep, d['value'], d['roofline']['avg_launch_ms'], p['ms_per_step'], p['actions_bit_equal'], p['bit_equal_to_rollout'], d.get('state_sha16'))"
  done
  # the unfused loop in C (pp3_rollout_policy's per-step policy + step launches) with the product library
  PP3_POLICY_UNFUSED=1 timeout -k 10 180 python3 bench.py --policy $POLICY --steps $STEPS --warmup 5 --no-cpu-baseline --no-extras > gpurun_out/ab_policy/unfused_$rep.log 2>&1 && \
    python3 -c "import json; d=json.loads(open('gpurun_out/ab_policy/unfused_$rep.log').read().strip().split('\n')[-1]); print('unfused-C', $rep, d['value'], d['roofline']['avg_launch_ms'], d.get('state_sha16'))"
done
