# round-5 job: blob pass A/B (hash_bench --no-ids, ABBA over libstl builds) + kernel trace
set -o pipefail
D=gpurun_out/${1:-r05k}; shift; mkdir -p $D
export TMPDIR=/tmp
for v in base "$@" "$@" base; do
  lib=""; [ "$v" != base ] && lib=build/ab/$v.so
  STL_LIB_PATH=$lib timeout -k 10 300 python -u tools/hash_bench.py --no-ids --reps 7 $([ "$v" != base ] && [ -n "$TIMING_ONLY" ] && echo --timing-only) >> $D/ab_$v.jsonl 2>>$D/ab.err || exit 1
  echo "$v $(tail -1 $D/ab_$v.jsonl | python -c 'import json,sys; d=json.load(sys.stdin); print(d["tx_hash"]["ms"], d["tx_blob"]["ms"])')"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof -o run -- python3 -u tools/hash_bench.py --no-ids --reps 3 > $D/prof.log 2>&1 || exit 1
find $D/prof -name '*kernel_stats.csv' -exec cp {} $D/kernel_stats.csv \;
python3 - $D/kernel_stats.csv <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    print(r["Name"][:60], r["Calls"], r["AverageNs"])
PY
