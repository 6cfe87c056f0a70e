#!/bin/bash
# r05e: A/B of the merged RNG (LDS-stashed pair) and the balanced SYRK (per-role loops)
set -u
mkdir -p gpurun_out/r05e
LIBS="default nomerge default nomerge" STEPS=300 bash tools/gpu_ab_lib.sh 2>&1 | tee gpurun_out/r05e/ab_merge.txt || exit 3
LIBS="default nobal default nobal" STEPS=20 C5=1 BENCH_ARGS="--indep 0 --ecorr 0 --c5-steps 3" bash tools/gpu_ab_lib.sh 2>&1 | tee gpurun_out/r05e/ab_syrk.txt
