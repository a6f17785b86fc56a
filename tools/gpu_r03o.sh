#!/bin/bash
# Joint table (default, sub-positions in one loop body), joint with both
# entries prefetched and the body duplicated (junroll), two tables (nojoint):
# VALU instruction / wait counters (one --pmc pass each, serial kernels), then
# same-process exec A/B in rotating order.
set -o pipefail
OUT=r03o
mkdir -p gpurun_out/$OUT
export TMPDIR=/tmp
B="python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extra"
for v in base junroll nojoint; do
  lib=""; [ $v != base ] && lib=build/ab/$v.so
  STL_STREAMS=1 STL_LIB_PATH=$lib timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE -d gpurun_out/$OUT/pmc_$v -o run --output-format csv -- $B > gpurun_out/$OUT/pmc_$v.log 2>&1
  rc=$?; echo "pmc $v rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
for v in base junroll nojoint nojoint junroll base base junroll nojoint; do
  lib=""; [ $v != base ] && lib=build/ab/$v.so
  STL_LIB_PATH=$lib timeout -k 10 200 python3 -u tools/exec_ab.py 20 3 s1=1,1,1,18 s2=1,1,2,18 \
    >> gpurun_out/$OUT/var_$v.jsonl 2> gpurun_out/$OUT/var_$v.err
  rc=$?; echo "variant $v rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
