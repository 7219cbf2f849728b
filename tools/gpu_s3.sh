#!/bin/bash
# round-2 session 3 check: GPU suite, driver bench, per-wave diag, 2-rank fallback rehearsal
OUT=gpurun_out/s3
mkdir -p $OUT
export PP3_REPORT_DIR=$OUT
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $OUT/gpu_tests.log 2>&1; rc=$?; echo tests_rc=$rc; tail -3 $OUT/gpu_tests.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $OUT/bench_driver.json 2>&1 || exit 1
tail -c 600 $OUT/bench_driver.json
PP3_DIAG_OUT=$OUT timeout -k 10 200 python tests/diag_phases.py > $OUT/phases.log 2>&1 || exit 1
head -40 $OUT/phases.log
# two ranks on the one GPU: RCCL refuses a duplicate device -> host-file barrier fallback
PP3_BENCH_DEVICE=0 timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 5 > $OUT/bench_2rank_1gpu.log 2>&1; echo two_rank_rc=$?
tail -c 1500 $OUT/bench_2rank_1gpu.log
