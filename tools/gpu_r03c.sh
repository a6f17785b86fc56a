#!/bin/bash
# Instruction-cache counters (serial kernels, then two streams) and the
# early-store phase-1 variant against the in-tree build, ABBA.
set -o pipefail
OUT=r03c
mkdir -p gpurun_out/$OUT
bash tools/icache_pmc.sh $OUT/ic_serial > gpurun_out/$OUT/ic_serial.log 2>&1
rc=$?; echo "icache serial rc=$rc"; cat gpurun_out/$OUT/ic_serial.log; [ $rc -eq 0 ] || exit $rc
STL_STREAMS=2 bash tools/icache_pmc.sh $OUT/ic_s2 > gpurun_out/$OUT/ic_s2.log 2>&1
rc=$?; echo "icache s2 rc=$rc"; [ $rc -eq 0 ] || exit $rc
for v in base early_def early_def base base early_def; do
  lib=""; [ $v != base ] && lib=build/ab/$v.so
  STL_LIB_PATH=$lib timeout -k 10 200 python3 -u tools/exec_ab.py 20 3 s1=1,1,1,18 s2=1,1,2,18 \
    >> gpurun_out/$OUT/var_$v.jsonl 2> gpurun_out/$OUT/var_$v.err
  rc=$?; echo "variant $v rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
