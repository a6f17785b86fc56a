#!/bin/bash
# Per-kernel times (rocprofv3 --kernel-trace --stats) of tools/perf_variant.py
# for each libstl variant.  usage: tools/ktrace.sh OUTDIR variant.so...
set -uo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1}; shift
mkdir -p $OUT
for so in "$@"; do
  b=$(basename $so .so)
  STL_LIB_PATH=$so timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/$b -o run --output-format csv -- python3 tools/perf_variant.py > $OUT/$b.log 2>&1 || { echo "FAIL $so"; tail -5 $OUT/$b.log; exit 1; }
  python3 - "$OUT/$b" <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        print("%-40s %6s calls  avg %9.3f ms" % (r["Name"][:40], r["Calls"], float(r["AverageNs"]) / 1e6))
PY
done
