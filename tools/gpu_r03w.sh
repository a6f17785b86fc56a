#!/bin/bash
# Host batch API, two streams of 64K chunks: one-lane phase 1 for chunks above
# pair_max (default: the chip is shared, so the cheaper kernel) vs the
# two-role phase 1 (midpair = previous build); GPU suite first.
set -o pipefail
OUT=r03w
mkdir -p gpurun_out/$OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/$OUT/pytest_gpu.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -2 gpurun_out/$OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for v in base midpair midpair base base midpair; do
  lib=""; [ $v != base ] && lib=build/ab/$v.so
  STL_LIB_PATH=$lib timeout -k 10 200 python3 -u tools/host_api_ab.py >> gpurun_out/$OUT/host_api_ab.log 2>&1
  rc=$?; echo "variant $v rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
grep "host API" gpurun_out/$OUT/host_api_ab.log
