#!/bin/bash
# Instruction-cache counters of the verify kernels: lists the counters the
# box's rocprofv3 offers, then one --pmc pass (never combined with tracing)
# with the SQC instruction-cache and SQ instruction-fetch counters found.
#   tools/icache_pmc.sh OUT [bench args...]
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-icache}; shift
mkdir -p $OUT
timeout -s KILL 60 rocprofv3 -L > $OUT/avail.txt 2>&1
echo "list rc=$?"
C=$(grep -oE '\b(SQC_ICACHE_(REQ|HITS|MISSES|MISSES_DUPLICATE)|SQ_IFETCH|SQ_IFETCH_LEVEL)\b' $OUT/avail.txt | sort -u | head -6 | tr '\n' ' ')
echo "counters: $C"
[ -n "$C" ] || exit 0
export STL_STREAMS=${STL_STREAMS:-1}
timeout -s KILL 90 rocprofv3 --pmc $C GRBM_GUI_ACTIVE -d $OUT/pmc -o run --output-format csv -- \
  python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-extra "$@" > $OUT/pmc.log 2>&1
echo "pmc rc=$?"
