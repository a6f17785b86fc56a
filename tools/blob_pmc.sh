#!/bin/bash
# Counters of the blob-path kernels (parse, hash) over tools/hash_bench.py,
# one rocprofv3 --pmc pass per group, never combined with tracing.
#   tools/blob_pmc.sh OUT
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-blobpmc}
mkdir -p $OUT
B="python3 tools/hash_bench.py --no-ids --reps 2"
pass() {
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" -d $OUT/$name -o run --output-format csv -- $B > $OUT/$name.log 2>&1 || return 1
}
pass insts SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_WAVES SQ_WAVE_CYCLES || exit 1
pass wait SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE || exit 1
pass fetch FETCH_SIZE || exit 1
python3 - $OUT <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.defaultdict(set)
for f in glob.glob(out + "/*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0]
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
        cnt[k].add(r["Dispatch_Id"])
for k, v in acc.items():
    if "blob" in k or "tx_hash" in k:
        print(k, {c: round(x / max(1, len(cnt[k]) // 3 or 1)) for c, x in sorted(v.items())})
PY
