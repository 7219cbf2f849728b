#!/bin/bash
# PMC of A/B kernel variants (via gpurun): for each ab/*.so, the kernel-trace pass and the SQ
# instruction-mix / wait pass of tools/gpu_profile.sh on the same bench command, then the summary
# (tools/summarize_profile.py) -> gpurun_out/$TAG/<variant>/.   tools/gpu_pmc_ab.sh TAG
set -e
TAG=${1:-pmc_ab}
ARGS="--steps 50 --warmup 5 --no-cpu-baseline --no-latency-floor --no-extras"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
for so in ab/*.so; do
  v=$(basename $so .so)
  OUT=gpurun_out/$TAG/$v
  mkdir -p $OUT
  PP3_LIB_PATH=$PWD/$so timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py $ARGS > $OUT/trace.log 2>&1
  PP3_LIB_PATH=$PWD/$so timeout -k 10 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY -d $OUT/pmc_sq -o run --output-format csv -- python3 bench.py $ARGS > $OUT/pmc_sq.log 2>&1
  python3 tools/summarize_profile.py $OUT > $OUT/summary.json
  python3 -c "
import json; d=json.load(open('$OUT/summary.json')); w=d['per_wave']
print('$v', 'launch_ns', d.get('kernel_avg_ns'), 'wait_any_frac', round(w['SQ_WAIT_ANY']/w['SQ_WAVE_CYCLES'],4), 'valu/wave/step', round(d['per_wave_per_step']['SQ_INSTS_VALU'],1))"
done
