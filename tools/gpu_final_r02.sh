#!/bin/bash
# round-end rehearsal: every -m gpu test, smoke(), bench, and the profile of the bench command
OUT=final_r02
bash tools/gpu_full.sh $OUT || exit $?
bash tools/profile.sh $OUT/prof > gpurun_out/$OUT/profile.log 2>&1
rc=$?; echo "profile rc=$rc"; tail -2 gpurun_out/$OUT/profile.log
exit $rc
