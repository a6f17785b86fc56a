#!/bin/bash
# Round 3 evidence + A/B pass (GIT_HEAD passed in by the caller):
#  1) rocprofv3 trace + FETCH/WRITE/SQ PMC passes of the bench command, kernels serial (tools/profile.sh)
#  2) VALU PMC passes (tools/valu_pmc.sh)
#  3) rocprofv3 kernel trace of the default execution (two streams, 2^18-signature chunks)
#  4) same-process A/B of the execution settings (tools/exec_ab.py, rotating/reversed order),
#     including phase 1 inside the main kernel (fused_prep 2)
#  5) build variants of the phase-1 kernel / whole kernel, one process each, ABBA
#  6) small-batch phases: DPP lane exchange (default) vs ds_bpermute (-DSTL_PAIR_SHFL), ABAB
set -o pipefail
OUT=r03b
mkdir -p gpurun_out/$OUT
export TMPDIR=/tmp
bash tools/profile.sh $OUT/prof > gpurun_out/$OUT/profile.log 2>&1
rc=$?; echo "profile rc=$rc"; [ $rc -eq 0 ] || exit $rc
bash tools/valu_pmc.sh $OUT/valu > gpurun_out/$OUT/valu.log 2>&1
rc=$?; echo "valu rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$OUT/trace_s2 -o run --output-format csv -- \
  python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-extra > gpurun_out/$OUT/trace_s2.log 2>&1
rc=$?; echo "trace_s2 rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 -u tools/exec_ab.py 20 6 s1=1,1,1,18 s2_18=1,1,2,18 s3_18=1,1,3,18 s2_19=1,1,2,19 \
  w1=2,1,1,18 w2_18=2,1,2,18 w2_17=2,1,2,17 w3_18=2,1,3,18 > gpurun_out/$OUT/exec_ab.json 2> gpurun_out/$OUT/exec_ab.err
rc=$?; echo "exec_ab rc=$rc"; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  order="base early early3 w3 early2 whole_paired"
  [ $r = 2 ] && order="whole_paired early2 w3 early3 early base"
  for v in $order; do
    lib=""; [ $v != base ] && lib=build/ab/$v.so
    set_w=1; [ $v = whole_paired ] && set_w=2
    STL_LIB_PATH=$lib timeout -k 10 200 python3 -u tools/exec_ab.py 20 3 s1=$set_w,1,1,18 s2=$set_w,1,2,18 \
      > gpurun_out/$OUT/var_${v}_$r.json 2> gpurun_out/$OUT/var_${v}_$r.err
    rc=$?; echo "variant $v $r rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
done
for r in 1 2; do
  for v in dpp shfl; do
    lib=""; [ $v = shfl ] && lib=build/ab/shfl.so
    STL_LIB_PATH=$lib timeout -k 10 200 python3 -u tools/phase_small.py --out gpurun_out/$OUT/phase_small_${v}_$r.json \
      > gpurun_out/$OUT/phase_small_${v}_$r.log 2>&1
    rc=$?; echo "phase_small $v $r rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
done
