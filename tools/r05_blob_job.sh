# round-5 job: blob-path parity tests, hash_bench (blob pass vs preimage hash), bench
set -o pipefail
D=gpurun_out/${1:-r05i}; mkdir -p $D
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_checksign_device.py tests/test_gpu_host_paths.py -m gpu -x -v --timeout 300 --timeout-method thread > $D/pytest.log 2>&1; rc=$?; tail -3 $D/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/hash_bench.py --no-ids --reps 5 > $D/hash_bench_noids.json 2>$D/hash_bench.err || exit 1; cat $D/hash_bench_noids.json
timeout -k 10 600 python -u bench.py > $D/bench.log 2>&1 || exit 1; echo bench-done
