# round-5 job: automatic-dedup row threshold A/B (ABBA over build/ab/*.so): config-1 one call, small ledgers
set -o pipefail
D=gpurun_out/${1:-r05z}; shift; mkdir -p $D
order=(base "$@")
for ((i=${#order[@]}-1; i>=0; i--)); do order+=("${order[$i]}"); done
for v in "${order[@]}"; do
  lib=""; [ "$v" != base ] && lib=build/ab/$v.so
  for n in 100000 200000; do
    STL_LIB_PATH=$lib timeout -k 10 300 python3 -u tools/host_blob_probe.py 10 $n device >> $D/dev_$v.jsonl 2>>$D/err.log || exit 1
    echo "$v $n $(tail -1 $D/dev_$v.jsonl | python3 -c 'import json,sys; print(json.load(sys.stdin)["ms_median"])')"
  done
  STL_LIB_PATH=$lib timeout -k 10 300 python3 -u tools/small_batch_probe.py 10 > $D/small_$v.log 2>>$D/err.log || exit 1
  grep -E "^(1000|4000|8000|19000) " $D/small_$v.log | sed "s/^/$v /" | cut -c1-120
done
