#!/bin/bash
mkdir -p gpurun_out/r02d
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -v -k dedup --timeout 300 --timeout-method thread > gpurun_out/r02d/pytest_dedup.log 2>&1
rc=$?; echo "dedup tests rc=$rc"; grep -E "PASSED|FAILED|Error" gpurun_out/r02d/pytest_dedup.log | tail -8
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u tools/report_configs.py --skip 4 --out gpurun_out/r02d/report_configs.json > gpurun_out/r02d/report.log 2>&1
rc=$?; echo "report rc=$rc"; tail -5 gpurun_out/r02d/report.log
exit $rc
