#!/bin/bash
# Hash-kernel profile (run on the GPU box from the repo root): kernel trace
# and one SQ counter pass over tools/hash_bench.py.
set -euo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-hashprof}
mkdir -p $OUT
timeout -k 10 200 python3 tools/hash_bench.py > $OUT/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 tools/hash_bench.py --reps 3 > $OUT/trace.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE -d $OUT/pmc_sq -o run --output-format csv -- python3 tools/hash_bench.py --reps 3 > $OUT/pmc_sq.log 2>&1
python3 tools/summarize_pmc.py $OUT tx_ > $OUT/pmc_summary.txt 2>&1 || true
cat $OUT/bench.json
echo hashprof-done
