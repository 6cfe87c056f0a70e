#!/bin/bash
# bench.py defaults + rocprofv3 kernel trace of the same command (the second half of
# tools/gpu_check.sh, for a rerun after the tests and smoke already passed).
set -u
OUT=gpurun_out
mkdir -p $OUT
export OPENBLAS_NUM_THREADS=1
timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > $OUT/bench.log 2>&1; rc=$?
echo "bench rc=$rc"; tail -3 $OUT/bench.log
[ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/prof -o run --output-format csv \
   -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline ${BENCH_ARGS:-} > $GRAFT_REPO_ROOT/$OUT/prof.log 2>&1; rc=$?
echo "rocprof rc=$rc"; tail -3 $GRAFT_REPO_ROOT/$OUT/prof.log
exit $rc
