#!/bin/bash
# r05d: full GPU suite on the merged-RNG / balanced-SYRK library, then A/B of both changes
set -u
bash tools/gpu_tests.sh r05d || exit $?
mkdir -p gpurun_out/r05d
LIBS="default nomerge default nomerge" STEPS=300 bash tools/gpu_ab_lib.sh 2>&1 | tee gpurun_out/r05d/ab_merge.txt || exit 3
LIBS="default nobal default nobal" STEPS=20 C5=1 BENCH_ARGS="--indep 0 --ecorr 0 --c5-steps 3" bash tools/gpu_ab_lib.sh 2>&1 | tee gpurun_out/r05d/ab_syrk.txt
