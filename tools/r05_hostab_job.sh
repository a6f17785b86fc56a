# round-5 job: host-path parity tests, then config-1 host API A/B (ABBA) against build/ab/*.so
set -o pipefail
D=gpurun_out/${1:-r05x}; shift; mkdir -p $D
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_host_paths.py -m gpu -x -v --timeout 300 --timeout-method thread > $D/pytest.log 2>&1; rc=$?; tail -3 $D/pytest.log; [ $rc -eq 0 ] || exit $rc
for v in base "$@" "$@" base; do
  lib=""; [ "$v" != base ] && lib=build/ab/$v.so
  for n in 100000 200000 1048576; do
    STL_LIB_PATH=$lib timeout -k 10 300 python3 -u tools/host_blob_probe.py 10 $n >> $D/host_$v.jsonl 2>>$D/host.err || exit 1
    echo "$v $n $(tail -1 $D/host_$v.jsonl | python3 -c 'import json,sys; print(json.load(sys.stdin)["ms_median"])')"
  done
done
