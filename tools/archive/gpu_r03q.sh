#!/bin/bash
# r03q: balanced fused sweep, 12-wave workgroups (3 waves on each SIMD of a CU) drawing 16 chains,
# each trio running one extra chain in thirds handed over through LDS (libpulsar_gibbs_bal.so):
# sweep parity on it first, then the headline / configs[2] A/B against the default library.
set -u
mkdir -p gpurun_out/r03q
export OPENBLAS_NUM_THREADS=1
GS_LIB_PATH=$PWD/pulsar_timing_gibbsspec_amd/libpulsar_gibbs_bal.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py \
  tests/test_gpu_indep.py tests/test_gpu_nf.py tests/test_gpu_big.py -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r03q/pytest.txt 2>&1
rc=$?; tail -3 gpurun_out/r03q/pytest.txt; [ $rc -eq 0 ] || exit $rc
LIBS="bal default bal default" CHAINS="4096" BENCH_ARGS="--ecorr 0 --host-stream 0" bash tools/gpu_ab_lib.sh
LIBS="bal default" CHAINS="3072 1000" BENCH_ARGS="--indep 0 --ecorr 0 --host-stream 0" bash tools/gpu_ab_lib.sh
