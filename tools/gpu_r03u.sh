#!/bin/bash
# Host batch API pipe-chunk size with two kernel streams: 2^17 (default) vs
# 2^18 (pc18) vs 2^16 (pc16), ABBA; then a kernel + memory-copy trace of the
# default's host-API calls (the timeline of chunks, copies and gaps).
set -o pipefail
OUT=r03u
mkdir -p gpurun_out/$OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_exec.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/$OUT/pytest_exec.log 2>&1
rc=$?; echo "exec tests rc=$rc"; tail -2 gpurun_out/$OUT/pytest_exec.log; [ $rc -eq 0 ] || exit $rc
for v in base pc18 pc16 pc16 pc18 base; do
  lib=""; [ $v != base ] && lib=build/ab/$v.so
  STL_LIB_PATH=$lib timeout -k 10 200 python3 -u tools/host_api_ab.py >> gpurun_out/$OUT/host_api_ab.log 2>&1
  rc=$?; echo "variant $v rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
grep "host API" gpurun_out/$OUT/host_api_ab.log
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/$OUT/trace -o run \
  -- python3 tools/host_api_ab.py > gpurun_out/$OUT/trace.log 2>&1
echo "trace rc=$?"
