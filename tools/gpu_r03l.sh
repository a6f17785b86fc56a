#!/bin/bash
# Timing-only: fewer stored multiples per lane table (STL_EXP_TABLE_ENTRIES:
# 6 -> 12 entries per lane, 1.5 KiB; 4 -> 1 KiB), the footprint and table-build
# cost a joint radix-4 table would have; ABBA against the current build.
set -o pipefail
OUT=r03l
mkdir -p gpurun_out/$OUT
for v in base e6 e4 base base e4 e6 base; do
  lib=""; [ $v != base ] && lib=build/ab/$v.so
  STL_AB_TIMING_ONLY=1 STL_LIB_PATH=$lib timeout -k 10 200 python3 -u tools/exec_ab.py 20 3 s1=1,1,1,18 s2=1,1,2,18 \
    >> gpurun_out/$OUT/var_$v.jsonl 2> gpurun_out/$OUT/var_$v.err
  rc=$?; echo "variant $v rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
