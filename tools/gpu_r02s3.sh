#!/bin/bash
# Session-3 evidence for the current build: rocprofv3 kernel trace + PMC passes
# of the bench command (tools/profile.sh), the VALU passes (tools/valu_pmc.sh)
# and the SURVEY section-8 configs report (CPU baselines included).
OUT=r02s3
mkdir -p gpurun_out/$OUT
bash tools/profile.sh $OUT/prof > gpurun_out/$OUT/profile.log 2>&1 || { echo "profile failed"; tail -5 gpurun_out/$OUT/profile.log; exit 1; }
echo profile-ok
bash tools/valu_pmc.sh $OUT/valu > gpurun_out/$OUT/valu.log 2>&1 || { echo "valu failed"; tail -5 gpurun_out/$OUT/valu.log; exit 1; }
echo valu-ok
timeout -k 10 1000 python -u tools/report_configs.py --skip 4 --out gpurun_out/$OUT/report_configs.json > gpurun_out/$OUT/report.log 2>&1
rc=$?; echo "report rc=$rc"; tail -3 gpurun_out/$OUT/report.log
exit $rc
