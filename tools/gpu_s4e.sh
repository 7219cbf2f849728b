#!/bin/bash
# Session 4: GPU suite (incl. the env-order test), then the pairing probe
OUT=gpurun_out/s4e
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $OUT/gpu_tests.log 2>&1; rc=$?; echo tests_rc=$rc; tail -30 $OUT/gpu_tests.log | grep -v "^$" | tail -12
[ $rc -eq 0 ] || exit 1
REPS=3 timeout -k 10 300 python3 tools/order_probe.py > $OUT/order_probe.jsonl 2>&1 || exit 1
cat $OUT/order_probe.jsonl
