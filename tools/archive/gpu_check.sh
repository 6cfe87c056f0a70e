#!/bin/bash
# One GPU session: parity tests, smoke, bench, rocprofv3 kernel trace.
# The library is built beforehand on the CPU container (it travels in-tree).
# Every GPU step has its own time limit; a crash/timeout/abort ends the script.
set -u
OUT=gpurun_out
mkdir -p $OUT
export OPENBLAS_NUM_THREADS=1
test -f pulsar_timing_gibbsspec_amd/libpulsar_gibbs.so || { echo "libpulsar_gibbs.so missing: build first"; exit 2; }
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }   # 1 = test/assert failure, not a fault
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ${PYTEST_ARGS:-} > $OUT/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -30 $OUT/pytest_gpu.log
ok $rc || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1; rc=$?
echo "smoke rc=$rc"; tail -5 $OUT/smoke.log
ok $rc || exit $rc
[ "${BENCH:-1}" = "1" ] || exit 0
timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > $OUT/bench.log 2>&1; rc=$?
echo "bench rc=$rc"; tail -3 $OUT/bench.log
[ $rc -eq 0 ] || exit $rc
if [ "${PROFILE:-1}" = "1" ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/prof -o run --output-format csv \
     -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline ${BENCH_ARGS:-} > $GRAFT_REPO_ROOT/$OUT/prof.log 2>&1; rc=$?
  echo "rocprof rc=$rc"; tail -3 $GRAFT_REPO_ROOT/$OUT/prof.log
fi
