# round-5 job: hash-path parity tests, then hash_bench A/B against build/ab/prev.so + kernel trace
set -o pipefail
D=gpurun_out/${1:-r05q}; mkdir -p $D
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_checksign_device.py -k "blob or hash or checksign or tx_" -m gpu -x -v --timeout 300 --timeout-method thread > $D/pytest.log 2>&1; rc=$?; tail -3 $D/pytest.log; [ $rc -eq 0 ] || exit $rc
bash tools/r05_blobab.sh ${1:-r05q} prev
