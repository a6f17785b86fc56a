#!/bin/bash
# Hash-kernel profile (trace + SQ counters + VALUBusy) on the config-5 shape.
set -o pipefail
OUT=r03f
mkdir -p gpurun_out/$OUT
bash tools/hash_prof.sh $OUT/hash > gpurun_out/$OUT/hash_prof.log 2>&1
rc=$?; echo "hash_prof rc=$rc"; tail -12 gpurun_out/$OUT/hash_prof.log; [ $rc -eq 0 ] || exit $rc
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc VALUBusy -d gpurun_out/$OUT/hash/pmc_busy -o run --output-format csv -- python3 tools/hash_bench.py --reps 3 > gpurun_out/$OUT/hash/pmc_busy.log 2>&1
echo "busy rc=$?"
