#!/bin/bash
# same-box A/B: table build with even multiples by doubling (dbl) vs HEAD (new), interleaved twice
OUT=r02h
bash tools/gpu_ab_r02.sh $OUT/a build/ab/new.so build/ab/dbl.so && bash tools/gpu_ab_r02.sh $OUT/b build/ab/dbl.so build/ab/new.so
