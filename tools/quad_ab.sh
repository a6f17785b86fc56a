set -o pipefail
D=gpurun_out/r04y; mkdir -p $D
for q in 0 1 2 4; do
  PROBE_QUAD=$q PROBE_SIZES=6000,8192,12000,16384,24000,32768 timeout -k 10 300 python3 -u tools/small_batch_probe.py 30 > $D/probe_q$q.log 2>&1 || exit $?
  echo q$q done
done
