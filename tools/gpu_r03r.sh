#!/bin/bash
# Joint table with LDS entry buffers filled a sub-position ahead by
# global_load_lds (default) vs the joint loop reading entries into VGPRs two
# doublings ahead (joint_vgpr, the previous default) vs two tables (nojoint):
# GPU suite on the default, ABBA exec A/B, one bench line.
set -o pipefail
OUT=r03r
mkdir -p gpurun_out/$OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/$OUT/pytest_gpu.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -2 gpurun_out/$OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for v in base joint_vgpr nojoint nojoint joint_vgpr base base joint_vgpr nojoint; do
  lib=""; [ $v != base ] && lib=build/ab/$v.so
  STL_LIB_PATH=$lib timeout -k 10 200 python3 -u tools/exec_ab.py 20 3 s1=1,1,1,18 s2=1,1,2,18 \
    >> gpurun_out/$OUT/var_$v.jsonl 2> gpurun_out/$OUT/var_$v.err
  rc=$?; echo "variant $v rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 400 python -u bench.py --no-extra > gpurun_out/$OUT/bench.log 2>&1; echo "bench rc=$?"; tail -c 600 gpurun_out/$OUT/bench.log
