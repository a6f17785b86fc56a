#!/bin/bash
# Profiling recipe (run on the GPU box from the repo root):
#   1) rocprofv3 --kernel-trace --stats of bench.py (per-kernel average times),
#   2) separate --pmc passes, never combined with tracing: FETCH_SIZE,
#      WRITE_SIZE, SQ instruction/occupancy counters + GRBM clock.
# tools/summarize_profile.py writes OUT/summary.json and, with --traffic,
# profiles/traffic_latest.json (HBM bytes per verify launch, read by bench.py).
set -euo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-prof}
mkdir -p $OUT
# STL_STREAMS=1: each verify call runs its kernels one after another on one
# stream (1M-signature chunks), so every kernel's duration and counters are its
# own -- the launches the bench's phase clock times
export STL_STREAMS=1 STL_EXEC_NOTE="STL_STREAMS=1 (kernels serial, 2^20-signature chunks)"
B="python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-extra"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- $B > $OUT/trace_bench.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o run --output-format csv -- $B > $OUT/pmc_fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o run --output-format csv -- $B > $OUT/pmc_write.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_LDS GRBM_GUI_ACTIVE -d $OUT/pmc_sq -o run --output-format csv -- $B > $OUT/pmc_sq.log 2>&1
python3 tools/summarize_profile.py $OUT --traffic > $OUT/summary.log && echo profile-done
