#!/bin/bash
# r03n: headline launch time against the chain count (3072 = one round of 3 waves/SIMD on 1024 SIMDs)
set -u
export OPENBLAS_NUM_THREADS=1
LIBS=default CHAINS="3072 4096 6144 2048 1024" BENCH_ARGS="--indep 0 --ecorr 0 --host-stream 0" bash tools/gpu_ab_lib.sh
