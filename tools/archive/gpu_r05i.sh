#!/bin/bash
set -u
bash tools/gpu_tests.sh r05i tests/test_gpu_ecorr.py || exit $?
mkdir -p gpurun_out/r05i
LIBS="default eclibm default eclibm" STEPS=50 BENCH_ARGS="--indep 0" bash tools/gpu_ab_lib.sh 2>&1 | tee gpurun_out/r05i/ab_ecorr.txt
