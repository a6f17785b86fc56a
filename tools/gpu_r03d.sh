#!/bin/bash
# GPU suite on the current build, then the table-build change (mixed
# additions + affine doubling) against the previous build (early store only), ABBA.
set -o pipefail
OUT=r03d
bash tools/gpu_full.sh $OUT || exit $?
for v in base early_def early_def base base early_def early_def base; do
  lib=""; [ $v != base ] && lib=build/ab/$v.so
  STL_LIB_PATH=$lib timeout -k 10 200 python3 -u tools/exec_ab.py 20 3 s1=1,1,1,18 s2=1,1,2,18 \
    >> gpurun_out/$OUT/var_$v.jsonl 2> gpurun_out/$OUT/var_$v.err
  rc=$?; echo "variant $v rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
