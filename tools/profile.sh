#!/bin/bash
# Round-1 profiling recipe (run on the GPU box from the repo root).
# 1) kernel-trace + stats of the bench, 2) separate PMC passes (FETCH_SIZE,
# WRITE_SIZE, SQ counters) -- never combined with tracing, one block per pass.
set -euo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-prof}
mkdir -p $OUT
B="python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline"
rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- $B > $OUT/trace_bench.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/pmc_fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/pmc_write.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE -d $OUT/pmc_sq -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/pmc_sq.log 2>&1
python3 tools/summarize_profile.py $OUT > $OUT/summary.log && echo profile-done
