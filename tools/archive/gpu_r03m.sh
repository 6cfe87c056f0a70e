#!/bin/bash
# r03m: issue-priority knobs of the fused sweep at 3 waves/SIMD (headline A/B, two passes)
set -u
export OPENBLAS_NUM_THREADS=1
LIBS="default d3 s2 u1 r1 default d3 s2 u1 r1" bash tools/gpu_ab_lib.sh
