#!/bin/bash
# One GPU call: the new host-path tests, the parity suite, the bench.
# Stops at the first step that did not end normally (pytest rc 0/1 only).
mkdir -p gpurun_out/r02a
timeout -k 10 600 python -u -m pytest tests/test_gpu_host_paths.py -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/r02a/pytest_new.log 2>&1
rc=$?; echo "new tests rc=$rc"; tail -5 gpurun_out/r02a/pytest_new.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r02a/pytest_old.log 2>&1
rc=$?; echo "old tests rc=$rc"; tail -3 gpurun_out/r02a/pytest_old.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u bench.py > gpurun_out/r02a/bench.log 2>&1
rc=$?; echo "bench rc=$rc"
tail -1 gpurun_out/r02a/bench.log | cut -c1-700
exit $rc
