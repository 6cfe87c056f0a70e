#!/bin/bash
# r03z2 closing check after the k_bdraw priority change: every GPU test, smoke, the driver's bench
# command, then the rocprof kernel trace of the bench.
set -u
export OPENBLAS_NUM_THREADS=1
bash tools/gpu_full.sh r03z2 || exit $?
bash tools/gpu_prof_trace.sh r03z2 || exit $?
