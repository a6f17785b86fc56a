#!/bin/bash
# A/B timing on the GPU box: microbenchmarks + verify-kernel time per libstl variant.
# usage: tools/gpu_ab.sh OUTDIR variant.so...
set -uo pipefail
OUT=gpurun_out/${1}; shift
mkdir -p $OUT
for mb in tools/microbench/isarate tools/microbench/isarate_v2; do
  if [ -x $mb ]; then timeout -k 10 120 $mb > $OUT/$(basename $mb).txt 2>&1 || { echo "FAIL $mb"; exit 1; }; fi
done
for so in "$@"; do
  STL_LIB_PATH=$so timeout -k 10 180 python3 tools/perf_variant.py >> $OUT/ab.txt 2>&1 || { echo "FAIL $so"; cat $OUT/ab.txt; exit 1; }
done
cat $OUT/*.txt
