#!/bin/bash
# Two-lanes-per-signature small-batch path: its parity test, the whole GPU
# suite, smoke, bench, and the latency A/B (pair vs STL_ONE_LANE).
OUT=gpurun_out/${1:-pair}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 240 --timeout-method thread -k "pair or ragged or golden or chunk" > $OUT/pytest_pair.log 2>&1
rc=$?; echo "pair tests rc=$rc"; tail -3 $OUT/pytest_pair.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/phase_small.py --out $OUT/phase_small.json > $OUT/phase_small.log 2>&1
rc=$?; echo "phases rc=$rc"; cat $OUT/phase_small.log | grep -v amdgpu.ids
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/latency.py --out $OUT/latency.json > $OUT/latency.log 2>&1
rc=$?; echo "latency rc=$rc"
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_full.sh ${1:-pair}/full
