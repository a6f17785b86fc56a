# round-5 job: kernel traces of hash_bench under timing-only parse variants
set -o pipefail
D=gpurun_out/${1:-r05r}; shift; mkdir -p $D
export TMPDIR=/tmp
for v in base "$@"; do
  lib=""; [ "$v" != base ] && lib=build/ab/$v.so
  STL_LIB_PATH=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof_$v -o run -- python3 -u tools/hash_bench.py --no-ids --reps 3 --timing-only > $D/prof_$v.log 2>&1 || exit 1
  f=$(find $D/prof_$v -name '*kernel_stats.csv' | head -1)
  python3 - $f $v <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "blob" in r["Name"] or "tx_hash" in r["Name"]:
        print(sys.argv[2], r["Name"][:40], r["Calls"], round(float(r["AverageNs"]) / 1000, 1), "us")
PY
done
