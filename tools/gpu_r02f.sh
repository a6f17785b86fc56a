#!/bin/bash
# dedup parity (wide / 9-entry / per-lane key tables), then the SURVEY-config
# report with the current build (phase splits included)
OUT=gpurun_out/r02f
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -v -k dedup --timeout 300 --timeout-method thread > $OUT/pytest_dedup.log 2>&1
rc=$?; echo "dedup tests rc=$rc"; grep -E "PASSED|FAILED|Error" $OUT/pytest_dedup.log | tail -8
[ $rc -eq 0 ] || exit $rc
timeout -k 10 1000 python -u tools/report_configs.py --out $OUT/report_configs.json > $OUT/report.log 2>&1
rc=$?; echo "report rc=$rc"; tail -3 $OUT/report.log
exit $rc
