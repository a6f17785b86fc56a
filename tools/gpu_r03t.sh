#!/bin/bash
# Host batch API with odd chunks' kernels on a second stream (default) vs one
# kernel stream (host1 = the previous build): GPU suite, ABAB host-API rates.
set -o pipefail
OUT=r03t
mkdir -p gpurun_out/$OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/$OUT/pytest_gpu.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -2 gpurun_out/$OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for v in base host1 host1 base base host1; do
  lib=""; [ $v != base ] && lib=build/ab/$v.so
  STL_LIB_PATH=$lib timeout -k 10 200 python3 -u tools/host_api_ab.py >> gpurun_out/$OUT/host_api_ab.log 2>&1
  rc=$?; echo "variant $v rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
cat gpurun_out/$OUT/host_api_ab.log
