#!/bin/bash
# r03v: final check of the committed tree: every GPU test, smoke, the driver's bench command.
set -u
export OPENBLAS_NUM_THREADS=1
bash tools/gpu_full.sh r03v || exit $?
