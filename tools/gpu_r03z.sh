#!/bin/bash
# Kernel trace of the bench's default device-resident execution (two streams
# of 2^18-signature chunks): where each chunk's kernels start and end, and
# whether the small fallback kernel waits for the other stream's main kernel.
set -o pipefail
OUT=r03z
mkdir -p gpurun_out/$OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/$OUT/trace -o run \
  -- python3 tools/exec_ab.py 10 1 s2=1,1,2,18 > gpurun_out/$OUT/trace.log 2>&1
echo "trace rc=$?"
