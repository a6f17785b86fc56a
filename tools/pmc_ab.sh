#!/bin/bash
# SQ counter pass per libstl variant (one rocprofv3 --pmc pass each; no tracing).
# usage: tools/pmc_ab.sh OUTDIR variant.so...
set -uo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1}; shift
mkdir -p $OUT
CNT="${CNT:-SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU}"
for so in "$@"; do
  b=$(basename $so .so)
  STL_LIB_PATH=$so N=${N:-1048576} timeout -s KILL 90 rocprofv3 --pmc $CNT -d $OUT/$b -o run --output-format csv -- python3 tools/perf_variant.py > $OUT/$b.log 2>&1 || { echo "FAIL $so"; tail -5 $OUT/$b.log; exit 1; }
done
python3 tools/summarize_pmc.py $OUT
