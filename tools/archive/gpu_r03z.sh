#!/bin/bash
# r03z closing check: every GPU test, smoke, the driver's bench command (CPU baselines included).
set -u
export OPENBLAS_NUM_THREADS=1
bash tools/gpu_full.sh r03z || exit $?
