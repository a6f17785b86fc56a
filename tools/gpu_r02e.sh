#!/bin/bash
# phase-timing tests, bench (live phase events), and the profile of the same bench command
OUT=gpurun_out/r02e
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_host_paths.py -m gpu -x -v -k "phase or stats" --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "PASSED|FAILED|Error" $OUT/pytest.log | tail -5
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py > $OUT/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 $OUT/bench.log | cut -c1-300
[ $rc -eq 0 ] || exit $rc
bash tools/profile.sh r02e/prof > $OUT/profile.log 2>&1
rc=$?; echo "profile rc=$rc"; tail -2 $OUT/profile.log
exit $rc
