#!/bin/bash
# Occupancy probe on the GPU box (via gpurun): tools/occ_probe.py for each ab/<name>.so given,
# at the env counts given.   tools/gpu_occ.sh TAG "base alias2 alias3" 4096 6144 8192
TAG=$1; LIBS=$2; shift 2
OUT=gpurun_out/$TAG
mkdir -p $OUT
for rep in 1 2; do
  for lib in $LIBS; do
    PP3_LIB_PATH=$PWD/ab/$lib.so timeout -k 10 200 python3 tools/occ_probe.py "$@" >> $OUT/occ.jsonl 2>> $OUT/occ.err || { tail $OUT/occ.err; exit 1; }
  done
done
cat $OUT/occ.jsonl
