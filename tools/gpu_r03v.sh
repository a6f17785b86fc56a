#!/bin/bash
# Host batch API pipe-chunk size with two kernel streams: 2^16 (default) vs
# 2^15 (pc15) vs 2^17 (pc17), ABBA, with 2^16 the default now; then a kernel + memory-copy trace of the
# default's host-API calls (the timeline of chunks, copies and gaps).
set -o pipefail
OUT=r03v
mkdir -p gpurun_out/$OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_exec.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/$OUT/pytest_exec.log 2>&1
rc=$?; echo "exec tests rc=$rc"; tail -2 gpurun_out/$OUT/pytest_exec.log; [ $rc -eq 0 ] || exit $rc
for v in base pc15 pc17 pc17 pc15 base; do
  lib=""; [ $v != base ] && lib=build/ab/$v.so
  STL_LIB_PATH=$lib timeout -k 10 200 python3 -u tools/host_api_ab.py >> gpurun_out/$OUT/host_api_ab.log 2>&1
  rc=$?; echo "variant $v rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
grep "host API" gpurun_out/$OUT/host_api_ab.log
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/$OUT/trace -o run \
  -- python3 tools/host_api_ab.py > gpurun_out/$OUT/trace.log 2>&1
echo "trace rc=$?"
timeout -k 10 600 python3 -u tools/report_configs.py --out gpurun_out/$OUT/report_configs.json > gpurun_out/$OUT/report_configs.log 2>&1
echo "report rc=$?"
