#!/bin/bash
# Session 4: loop-alignment variants (same instructions + s_nop padding) vs HEAD, interleaved
OUT=gpurun_out/s4i
mkdir -p $OUT
REPS=3 STEPS=20 timeout -k 10 500 tools/ab_bench.sh > $OUT/ab20.txt 2>&1 || exit 1
cat $OUT/ab20.txt
REPS=2 STEPS=200 timeout -k 10 500 tools/ab_bench.sh > $OUT/ab200.txt 2>&1 || exit 1
cat $OUT/ab200.txt
