#!/bin/bash
# r04o: every GPU test, smoke, the driver's bench command, then the rocprof kernel trace of the bench.
set -u
export OPENBLAS_NUM_THREADS=1
bash tools/gpu_full.sh r04o || exit $?
bash tools/gpu_prof_trace.sh r04o || exit $?
