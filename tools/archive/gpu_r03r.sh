#!/bin/bash
# r03r: the hand-off sweep chosen by the launch cost model (default): every GPU test, smoke, the
# driver's bench command, then the rocprof kernel trace of the bench.
set -u
export OPENBLAS_NUM_THREADS=1
bash tools/gpu_full.sh r03r || exit $?
bash tools/gpu_prof_trace.sh r03r || exit $?
