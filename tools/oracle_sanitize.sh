#!/bin/bash
# The CPU oracle (test infrastructure) under AddressSanitizer + UndefinedBehaviorSanitizer: build
# both precisions of oracle/pp3_oracle.c instrumented into oracle/_asan/, then run every CPU test
# that drives the oracle with it (oracle.lib() reads PP3_ORACLE_DIR), halting on the first report.
#   tools/oracle_sanitize.sh            (CPU only, ~1 min)
set -e
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
OUT=$ROOT/oracle/_asan
mkdir -p $OUT
SAN="-O1 -g -fPIC -shared -std=c11 -fopenmp -fsanitize=address,undefined -fno-omit-frame-pointer"
gcc $SAN -DREAL=double -o $OUT/liboracle64.so $ROOT/oracle/pp3_oracle.c -lm
gcc $SAN -DREAL=float -DORC_FLOAT -ffp-contract=off -o $OUT/liboracle32.so $ROOT/oracle/pp3_oracle.c -lm
TESTS=$(cd $ROOT && grep -l "from oracle import\|import oracle" tests/test_*.py | grep -v "tests/test_gpu_")
cd $ROOT
ASAN_OPTIONS=detect_leaks=0:halt_on_error=1 UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1 \
  PP3_ORACLE_DIR=$OUT LD_PRELOAD=$(gcc -print-file-name=libasan.so):$(gcc -print-file-name=libubsan.so) \
  python -m pytest $TESTS -x -q -m "not gpu" -p no:cacheprovider
