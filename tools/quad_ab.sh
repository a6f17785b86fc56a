# A/B of the lane-group main kernels for small chunks (STL_TUNE_QUAD: bit 0
# quads, bit 1 duos; 0 = lane pairs): tools/small_batch_probe.py per setting.
set -o pipefail
D=gpurun_out/${1:-quad_ab}; mkdir -p $D
for q in 0 1 3; do
  PROBE_QUAD=$q PROBE_SIZES=${2:-4000,8192,10000,12000,16384,20000} timeout -k 10 300 python3 -u tools/small_batch_probe.py 30 > $D/probe_q$q.log 2>&1 || exit $?
  echo q$q done
done
