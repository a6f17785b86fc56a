#!/bin/bash
# Joint radix-4 per-lane table (default) vs two radix-16 tables (-DSTL_NO_JOINT):
# GPU suite on the new build, then ABBA exec A/B and a bench line.
set -o pipefail
OUT=${OUT:-r03m}
mkdir -p gpurun_out/$OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/$OUT/pytest_gpu.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -2 gpurun_out/$OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for v in base nojoint nojoint base base nojoint nojoint base; do
  lib=""; [ $v != base ] && lib=build/ab/$v.so
  STL_LIB_PATH=$lib timeout -k 10 200 python3 -u tools/exec_ab.py 20 3 s1=1,1,1,18 s2=1,1,2,18 \
    >> gpurun_out/$OUT/var_$v.jsonl 2> gpurun_out/$OUT/var_$v.err
  rc=$?; echo "variant $v rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 300 python3 -u bench.py > gpurun_out/$OUT/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/$OUT/bench.log | cut -c1-200; exit $rc
