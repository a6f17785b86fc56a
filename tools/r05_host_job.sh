# round-5 job: config-1 host API timeline (plain timing, then kernel + copy trace)
set -o pipefail
D=gpurun_out/${1:-r05w}; mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 300 python3 -u tools/host_blob_probe.py 10 > $D/host.json 2> $D/host.err || exit 1
cat $D/host.json
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $D/trace -o run -- python3 -u tools/host_blob_probe.py 4 > $D/trace.log 2>&1 || exit 1
ls $D/trace
