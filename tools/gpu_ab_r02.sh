#!/bin/bash
# same-box A/B: per-kernel times of each variant (rocprofv3 kernel trace)
OUT=$1; shift
bash tools/ktrace.sh $OUT "$@" 2>&1 | grep -E "verify_|FAIL"
