#!/bin/bash
# Round 3: suite + smoke + bench on HEAD, then the rocprofv3 trace / PMC passes
# (traffic and VALU) of the same bench command, then the small-batch phases.
OUT=r03a
bash tools/gpu_full.sh $OUT || exit $?
bash tools/profile.sh $OUT/prof > gpurun_out/$OUT/profile.log 2>&1
rc=$?; echo "profile rc=$rc"; tail -2 gpurun_out/$OUT/profile.log; [ $rc -eq 0 ] || exit $rc
bash tools/valu_pmc.sh $OUT/valu > gpurun_out/$OUT/valu.log 2>&1
rc=$?; echo "valu rc=$rc"; tail -2 gpurun_out/$OUT/valu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/phase_small.py --out gpurun_out/$OUT/phase_small.json > gpurun_out/$OUT/phase_small.log 2>&1
rc=$?; echo "phase_small rc=$rc"; exit $rc
