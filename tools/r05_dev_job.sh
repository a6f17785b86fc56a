# round-5 job: config-1 device-resident one call, timing then kernel trace
set -o pipefail
D=gpurun_out/${1:-r05y}; mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 300 python3 -u tools/host_blob_probe.py 10 100000 device > $D/dev.json 2> $D/dev.err || exit 1
cat $D/dev.json
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $D/trace -o run -- python3 -u tools/host_blob_probe.py 4 100000 device > $D/trace.log 2>&1 || exit 1
