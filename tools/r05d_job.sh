# round-5 job: long-mode hash parity tests, then small-ledger latency A/B (STL_TUNE_LONG_HASH 0 / 8)
set -o pipefail
D=gpurun_out/${1:-r05d}; mkdir -p $D
timeout -k 10 600 python -u -m pytest tests/test_gpu_checksign_device.py -m gpu -x -v --timeout 300 --timeout-method thread > $D/pytest.log 2>&1; rc=$?; tail -3 $D/pytest.log; [ $rc -eq 0 ] || exit $rc
for L in 0 8 8 0; do PROBE_LONG=$L PROBE_SIZES=1000,4000,8000,19000 timeout -k 10 300 python -u tools/small_batch_probe.py 20 > $D/probe_long${L}_$(date +%s%N).json 2>>$D/probe.err || exit 1; echo "probe long=$L done"; done
ls $D
[ -n "$2" ] && { timeout -k 10 400 python -u tools/hash_bench.py --no-ids --reps 5 > $D/hash_bench_noids.json 2>$D/hash_bench.err || exit 1; cat $D/hash_bench_noids.json; }
