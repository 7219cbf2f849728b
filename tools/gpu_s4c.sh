#!/bin/bash
# Session 4: FP32 instruction-mix PMC pass, then the driver's bench command (reads the new fp32 figure)
OUT=gpurun_out/s4c
mkdir -p $OUT
tools/gpu_flops.sh s4flops || exit 1
python3 tools/summarize_flops.py gpurun_out/s4flops --commit gpurun_out/s4c/r02_v14 > /dev/null || exit 1
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $OUT/bench_driver.json 2>&1 || exit 1
tail -c 1500 $OUT/bench_driver.json | head -c 1500
