#!/bin/bash
# r03o: balanced fused sweep (6-wave workgroups, 8 chains each, the extra chains in thirds handed
# over through LDS): sweep parity first, then the headline / configs[2] A/B against nobal.
set -u
mkdir -p gpurun_out/r03o
export OPENBLAS_NUM_THREADS=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_indep.py tests/test_gpu_nf.py tests/test_gpu_big.py \
  -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03o/pytest.txt 2>&1
rc=$?; tail -3 gpurun_out/r03o/pytest.txt; [ $rc -eq 0 ] || exit $rc
LIBS="default nobal default nobal" CHAINS="4096" BENCH_ARGS="--ecorr 0 --host-stream 0" bash tools/gpu_ab_lib.sh
LIBS="default nobal" CHAINS="3072 1000" BENCH_ARGS="--indep 0 --ecorr 0 --host-stream 0" bash tools/gpu_ab_lib.sh
