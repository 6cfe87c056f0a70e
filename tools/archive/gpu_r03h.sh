#!/bin/bash
# r03h: k_bdraw (CURN line) A/B: chain-group loop 4 / 8, tiled model staging, both; parity of the
# tiled loop build on the PTA fixtures first.
set -u
mkdir -p gpurun_out/r03h
export OPENBLAS_NUM_THREADS=1
for v in l4t l8t; do
  GS_LIB_PATH=$PWD/pulsar_timing_gibbsspec_amd/libpulsar_gibbs_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_grid_pta.py \
    tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03h/pytest_$v.txt 2>&1
  rc=$?; echo "$v parity rc=$rc"; tail -2 gpurun_out/r03h/pytest_$v.txt; [ $rc -eq 0 ] || exit $rc
done
LIBS="${PLIBS:-default loop4 loop8 l1t l4t l8t default l4t l8t}" PTA=curn bash tools/gpu_ab_pta.sh
