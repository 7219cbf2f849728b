#!/bin/bash
# A/B timing of kernel variants on the GPU box (via gpurun): each .so under ab/ is benched
# twice, interleaved (v1 v2 ... v1 v2 ...), configs[1] bench line -> gpurun_out/ab/<tag>.log
set -e
mkdir -p gpurun_out/ab
for rep in 1 2; do
  for so in ab/*.so; do
    tag=$(basename $so .so)
    PP3_LIB_PATH=$PWD/$so timeout -k 10 120 python3 bench.py --steps 400 --warmup 20 --no-cpu-baseline > gpurun_out/ab/${tag}_$rep.log 2>&1
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/ab/${tag}_$rep.log').read().strip().split('\n')[-1]); print('$tag', $rep, d['value'], d['roofline']['avg_launch_ms'])"
  done
done
