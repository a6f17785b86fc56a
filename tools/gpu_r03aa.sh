#!/bin/bash
# Device-resident execution settings re-checked with the joint table (same
# process, rotating order): streams x chunk size.
set -o pipefail
OUT=r03aa
mkdir -p gpurun_out/$OUT
timeout -k 10 400 python3 -u tools/exec_ab.py 20 5 s2_18=1,1,2,18 s3_18=1,1,3,18 s2_17=1,1,2,17 s3_17=1,1,3,17 s4_16=1,1,4,16 s1=1,1,1,20 \
  > gpurun_out/$OUT/exec_ab.json 2> gpurun_out/$OUT/exec_ab.err
rc=$?; echo "exec_ab rc=$rc"; cat gpurun_out/$OUT/exec_ab.json | tr -d '\n ' | head -c 1500
