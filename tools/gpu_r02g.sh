#!/bin/bash
# same-box A/B of the bench path: HEAD build (old) vs the working tree (new), twice interleaved
OUT=r02g
bash tools/gpu_ab_r02.sh $OUT/a build/ab/old.so build/ab/new.so && bash tools/gpu_ab_r02.sh $OUT/b build/ab/new.so build/ab/old.so
