#!/bin/bash
# One parameterised GPU-box job (replaces the per-session gpu_r0*.sh scripts).
#
#   tools/gpujob.sh OUT STEP [STEP ...]
#
# Runs from the repo root on the GPU box; every step writes under
# gpurun_out/OUT and has its own time limit; the job stops at the first
# failing step (no retries).  Steps:
#   suite              pytest -m gpu (the round-end suite)
#   tests:F1,F2        pytest -m gpu on the named test files / node ids only
#   smoke              __graft_entry__.smoke()
#   bench              python bench.py (defaults: the driver's N = 1 line)
#   bench2             bench.py --gpus 2 --gather gloo (multi-rank rehearsal on one GPU)
#   profile            tools/profile.sh: kernel trace + FETCH/WRITE/SQ PMC passes
#   valu               tools/valu_pmc.sh: VALUBusy / INT64 / occupancy PMC passes
#   ab:K:R:V1,V2       ABBA of libstl builds build/ab/V.so ("base" = stellard_amd/libstl.so),
#                      tools/exec_ab.py K launches x R rotations per run, serial + 2-stream
#   hab:V1,V2          ABBA of the host batch API (tools/host_api_ab.py, PCIe included) over
#                      libstl builds build/ab/V.so ("base" = stellard_amd/libstl.so)
#   py:SCRIPT[:ARGS]   python3 tools/SCRIPT ARGS (comma-separated ARGS), stdout to OUT/SCRIPT.log
#   exec:N:K:R:SPECS   tools/exec_ab.py on N signatures, K launches x R rotations, settings
#                      SPECS (name=fused,queue,streams,log2 separated by +), to OUT/exec_N.json
#   abpy:SCRIPT:ARGS:V1,V2  ABBA of python3 tools/SCRIPT ARGS (comma-separated) over libstl
#                      builds build/ab/V.so ("base" = the product), each run's last stdout
#                      line appended to OUT/SCRIPT_V.jsonl (hash_bench.py, prep_probe.py,
#                      host_blob_probe.py, small_batch_probe.py)
#   trace:SCRIPT:ARGS  rocprofv3 --kernel-trace --memory-copy-trace of python3 tools/SCRIPT
#                      ARGS, CSVs under OUT/trace_SCRIPT
set -o pipefail
OUT=$1; shift
[ -n "$OUT" ] || { echo "usage: tools/gpujob.sh OUT STEP..."; exit 2; }
D=gpurun_out/$OUT
mkdir -p $D
export TMPDIR=/tmp

run() {  # run NAME SECONDS CMD...
  local name=$1 secs=$2; shift 2
  local t0=$(date +%s)
  timeout -k 10 $secs "$@" > $D/$name.log 2>&1
  local rc=$?
  echo "[$name] rc=$rc $(( $(date +%s) - t0 )) s"
  tail -2 $D/$name.log
  return $rc
}

for step in "$@"; do
  case $step in
    suite) run pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread || exit $? ;;
    tests:*)
      T=${step#tests:}
      run pytest_gpu_part 900 python -u -m pytest ${T//,/ } -m gpu -x -v --timeout 300 --timeout-method thread || exit $? ;;
    smoke) run smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" || exit $? ;;
    bench) run bench 600 python -u bench.py || exit $? ;;
    bench2) run bench_n2_rehearsal 600 python -u bench.py --gpus 2 --gather gloo --no-cpu-baseline || exit $? ;;
    profile) run profile 900 bash tools/profile.sh $OUT/prof || exit $? ;;
    valu) run valu 900 bash tools/valu_pmc.sh $OUT/valu || exit $? ;;
    ab:*)
      IFS=: read -r _ K R VS <<< "$step"
      IFS=, read -r -a vs <<< "$VS"
      order=("${vs[@]}")
      for ((i=${#vs[@]}-1; i>=0; i--)); do order+=("${vs[$i]}"); done
      for v in "${order[@]}" "${order[@]}"; do
        lib=""; [ "$v" != base ] && lib=build/ab/$v.so
        STL_LIB_PATH=$lib timeout -k 10 300 python3 -u tools/exec_ab.py $K $R s1=1,1,1,18 s2=1,1,2,18 \
          >> $D/var_$v.jsonl 2>> $D/var_$v.err
        rc=$?; echo "variant $v rc=$rc"; [ $rc -eq 0 ] || exit $rc
      done ;;
    hab:*)
      IFS=, read -r -a vs <<< "${step#hab:}"
      order=("${vs[@]}")
      for ((i=${#vs[@]}-1; i>=0; i--)); do order+=("${vs[$i]}"); done
      for v in "${order[@]}"; do
        lib=""; [ "$v" != base ] && lib=build/ab/$v.so
        STL_LIB_PATH=$lib timeout -k 10 300 python3 -u tools/host_api_ab.py >> $D/hab.log 2>> $D/hab.err
        rc=$?; echo "host-api variant $v rc=$rc"; [ $rc -eq 0 ] || exit $rc
      done
      tail -$(( 2 * ${#vs[@]} )) $D/hab.log ;;
    exec:*)
      IFS=: read -r _ NS K R SP <<< "$step"
      N=$NS run exec_$NS 300 python3 -u tools/exec_ab.py $K $R ${SP//+/ } || exit $?
      cp $D/exec_$NS.log $D/exec_$NS.json ;;
    py:*)
      IFS=: read -r _ S A <<< "$step"
      run ${S%.py} 600 python3 -u tools/$S ${A//,/ } || exit $? ;;
    abpy:*)
      IFS=: read -r _ S A VS <<< "$step"
      IFS=, read -r -a vs <<< "$VS"
      order=("${vs[@]}")
      for ((i=${#vs[@]}-1; i>=0; i--)); do order+=("${vs[$i]}"); done
      for v in "${order[@]}"; do
        lib=""; [ "$v" != base ] && lib=build/ab/$v.so
        STL_LIB_PATH=$lib timeout -k 10 300 python3 -u tools/$S ${A//,/ } > $D/${S%.py}_run.out 2>> $D/${S%.py}.err
        rc=$?; echo "$S variant $v rc=$rc: $(tail -c 300 $D/${S%.py}_run.out | tail -1)"
        [ $rc -eq 0 ] || exit $rc
        cat $D/${S%.py}_run.out >> $D/${S%.py}_$v.out
        tail -1 $D/${S%.py}_run.out >> $D/${S%.py}_$v.jsonl
      done ;;
    trace:*)
      IFS=: read -r _ S A <<< "$step"
      run trace_${S%.py} 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv \
        -d $D/trace_${S%.py} -o run -- python3 -u tools/$S ${A//,/ } || exit $? ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "gpujob $OUT done"
