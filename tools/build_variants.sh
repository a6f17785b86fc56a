#!/bin/bash
# Build libstl variants for same-box A/B runs: tools/build_variants.sh NAME "FLAGS" [NAME "FLAGS" ...]
# Output build/ab/NAME.so (travels to the GPU box; build/ab is not gpurun-ignored).
set -e
cd "$(dirname "$0")/.."
mkdir -p build/ab
pids=()
while [ $# -ge 2 ]; do
  n=$1; f=$2; shift 2
  ( hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared $f -o build/ab/$n.so \
      stellard_amd/csrc/stl_kernels.hip stellard_amd/csrc/stl_api.cpp stellard_amd/csrc/stl_batcher.cpp \
      && echo "built $n" ) &
  pids+=($!)
done
for p in "${pids[@]}"; do wait $p; done
