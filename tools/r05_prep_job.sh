# round-5 job: prep / main phase split of timing-only libstl builds (ABBA)
set -o pipefail
D=gpurun_out/${1:-r05v}; shift; mkdir -p $D
export STL_STREAMS=1
for v in base "$@" "$@" base; do
  lib=""; [ "$v" != base ] && lib=build/ab/$v.so
  STL_LIB_PATH=$lib timeout -k 10 300 python3 -u tools/prep_probe.py 10 >> $D/prep_$v.jsonl 2>>$D/prep.err || exit 1
  echo "$v $(tail -1 $D/prep_$v.jsonl)"
done
