#!/bin/bash
# Round-3 evidence on the current build: GPU suite, smoke, bench, then the
# rocprofv3 trace / PMC passes (traffic, VALU) of the serial bench launches.
OUT=r03h
bash tools/gpu_full.sh $OUT || exit $?
bash tools/profile.sh $OUT/prof > gpurun_out/$OUT/profile.log 2>&1
rc=$?; echo "profile rc=$rc"; tail -2 gpurun_out/$OUT/profile.log; [ $rc -eq 0 ] || exit $rc
bash tools/valu_pmc.sh $OUT/valu > gpurun_out/$OUT/valu.log 2>&1
rc=$?; echo "valu rc=$rc"; tail -2 gpurun_out/$OUT/valu.log; exit $rc
