#!/bin/bash
# BASELINE.json configs report on the final round-3 build (joint table), and the two-rank bench
# rehearsal on the one GPU (gloo gather through host memory).
set -o pipefail
OUT=r03s
mkdir -p gpurun_out/$OUT
timeout -k 10 600 python3 -u tools/report_configs.py --out gpurun_out/$OUT/report_configs.json > gpurun_out/$OUT/report_configs.log 2>&1
rc=$?; echo "report rc=$rc"; tail -3 gpurun_out/$OUT/report_configs.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 -u bench.py --gpus 2 --gather gloo --no-cpu-baseline > gpurun_out/$OUT/bench_n2_rehearsal.log 2>&1
rc=$?; echo "n2 rc=$rc"; tail -1 gpurun_out/$OUT/bench_n2_rehearsal.log | cut -c1-300
exit $rc
