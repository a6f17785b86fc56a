#!/bin/bash
# Integer-VALU counters of the verify kernels (north_star: VALUBusy, VALU
# int-op rate, occupancy), one rocprofv3 --pmc pass per group, never combined
# with tracing.  Run on the GPU box from the repo root:  tools/valu_pmc.sh OUT
set -euo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-valu}
mkdir -p $OUT
# STL_STREAMS=1: each verify call runs its kernels one after another on one
# stream (1M-signature chunks), so every kernel's duration and counters are its
# own -- the launches the bench's phase clock times
export STL_STREAMS=1 STL_EXEC_NOTE="STL_STREAMS=1 (kernels serial, 2^20-signature chunks)"
B="python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-extra"
pass() {
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" -d $OUT/$name -o run --output-format csv -- $B > $OUT/$name.log 2>&1
}
pass int SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_IOPS SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVES GRBM_GUI_ACTIVE
pass busy VALUBusy
pass util VALUUtilization
pass occ OccupancyPercent
pass mocc MeanOccupancyPerActiveCU
python3 tools/summarize_valu.py $OUT > $OUT/summary.log && echo valu-pmc-done
