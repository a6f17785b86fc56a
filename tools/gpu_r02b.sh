#!/bin/bash
# Digest parity at full config sizes + single-call latency.
mkdir -p gpurun_out/r02b
timeout -k 10 900 python -u -m pytest tests/test_gpu_digests.py -m gpu -v -s --timeout 300 --timeout-method thread > gpurun_out/r02b/pytest_digests.log 2>&1
rc=$?; echo "digest tests rc=$rc"; grep -E "PASSED|FAILED|bitmap digest|Error|assert" gpurun_out/r02b/pytest_digests.log | tail -12
[ $rc -le 1 ] || exit $rc
timeout -k 10 600 python -u tools/latency.py --out gpurun_out/r02b/latency.json > gpurun_out/r02b/latency.log 2>&1
rc=$?; echo "latency rc=$rc"; tail -c 2500 gpurun_out/r02b/latency.log
exit $rc
