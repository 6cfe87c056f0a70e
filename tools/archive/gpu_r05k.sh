#!/bin/bash
set -u
bash tools/gpu_tests.sh r05k tests/test_gpu_big.py tests/test_gpu_white.py tests/test_gpu_ecorr.py || exit $?
mkdir -p gpurun_out/r05k
LIBS="default noglds default noglds" STEPS=20 C5=1 BENCH_ARGS="--indep 0 --ecorr 0 --c5-steps 3" bash tools/gpu_ab_lib.sh 2>&1 | tee gpurun_out/r05k/ab_syrk.txt
