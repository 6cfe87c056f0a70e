#!/bin/bash
# fast-math / exec-mask change: accuracy probe, GPU tests, headline A/B of the variants.
set -u
O=gpurun_out
mkdir -p $O
export OPENBLAS_NUM_THREADS=1
timeout -k 10 60 ./tools/probe/fastmath_probe > $O/fastmath_probe.json 2>&1 || { echo "probe failed"; cat $O/fastmath_probe.json; exit 3; }
cat $O/fastmath_probe.json
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -3 $O/pytest_gpu.log; grep -E "FAILED|Error" $O/pytest_gpu.log | head -10
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
LIBS="${LIBS:-old cur fm em}" REPS=${REPS:-2} bash tools/gpu_ab_variants.sh
