#!/bin/bash
# Session 4: dense_search marked cold (bitwise-neutral) vs HEAD, interleaved
OUT=gpurun_out/s4j
mkdir -p $OUT
REPS=4 STEPS=20 timeout -k 10 400 tools/ab_bench.sh > $OUT/ab20.txt 2>&1 || exit 1
cat $OUT/ab20.txt
REPS=2 STEPS=200 timeout -k 10 400 tools/ab_bench.sh > $OUT/ab200.txt 2>&1 || exit 1
cat $OUT/ab200.txt
