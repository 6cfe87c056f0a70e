#!/bin/bash
# Iteration loop on one box: tile parity tests, A/B bench of library variants, phase profiles.
# LIBS="default v1 ..." PHASES="phase phasev1" bash tools/gpu_iter.sh
set -u
mkdir -p gpurun_out
export OPENBLAS_NUM_THREADS=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_tile.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_tile.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
LIBS="${LIBS:-default}" CHAINS="${CHAINS:-4096}" bash tools/gpu_ab_lib.sh || exit 3
for ph in ${PHASES:-}; do
  echo "== $ph"
  GS_LIB_PATH=$PWD/pulsar_timing_gibbsspec_amd/libpulsar_gibbs_$ph.so timeout -k 10 120 python tools/phase_prof.py 2>/dev/null || exit 4
done
