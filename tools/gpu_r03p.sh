#!/bin/bash
# Joint table, software-pipelined over sub-positions (default) vs the joint
# loop-body version (jloop) vs two tables (nojoint): GPU suite on the default,
# then ABBA exec A/B, then I-cache counters of the default (its Straus loop is
# 64 KB).
set -o pipefail
OUT=r03p
mkdir -p gpurun_out/$OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/$OUT/pytest_gpu.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -2 gpurun_out/$OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for v in base jloop nojoint nojoint jloop base base jloop nojoint; do
  lib=""; [ $v != base ] && lib=build/ab/$v.so
  STL_LIB_PATH=$lib timeout -k 10 200 python3 -u tools/exec_ab.py 20 3 s1=1,1,1,18 s2=1,1,2,18 \
    >> gpurun_out/$OUT/var_$v.jsonl 2> gpurun_out/$OUT/var_$v.err
  rc=$?; echo "variant $v rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
bash tools/icache_pmc.sh $OUT/ic > gpurun_out/$OUT/ic.log 2>&1; echo "icache rc=$?"
