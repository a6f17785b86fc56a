#!/bin/bash
# Small-batch phase 1 as one two-role launch (verify_prep_pair_kernel) vs the
# previous build (scalar kernel, then the point-pair kernel): GPU suite on the
# new build, then phase_small ABAB and single-call latency of both.
set -o pipefail
OUT=${OUT:-r03i}
mkdir -p gpurun_out/$OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/$OUT/pytest_gpu.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -2 gpurun_out/$OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for v in new prev; do
    lib=""; [ $v = prev ] && lib=build/ab/prev.so
    STL_LIB_PATH=$lib timeout -k 10 200 python3 -u tools/phase_small.py --out gpurun_out/$OUT/phase_small_${v}_$r.json \
      > gpurun_out/$OUT/phase_small_${v}_$r.log 2>&1
    rc=$?; echo "phase_small $v $r rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
done
for v in new prev; do
  lib=""; [ $v = prev ] && lib=build/ab/prev.so
  STL_LIB_PATH=$lib timeout -k 10 300 python3 -u tools/latency.py --out gpurun_out/$OUT/latency_$v.json > gpurun_out/$OUT/latency_$v.log 2>&1
  rc=$?; echo "latency $v rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
