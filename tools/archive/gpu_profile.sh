#!/bin/bash
# rocprofv3 evidence for the bench's dominant kernel: kernel trace + stats, then
# FETCH_SIZE and WRITE_SIZE in separate --pmc passes (MI355X_MICROARCH.md §HBM).
set -u
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/prof_${TAG:-r01}
mkdir -p $OUT
export OPENBLAS_NUM_THREADS=1
test -f $R/pulsar_timing_gibbsspec_amd/libpulsar_gibbs.so || { echo "build first"; exit 2; }
ARGS="--no-cpu-baseline --pta none --config5 0 ${BENCH_ARGS:-}"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $R/bench.py $ARGS > $OUT/trace.log 2>&1; rc=$?
echo "trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- python3 $R/bench.py $ARGS > $OUT/pmc_fetch.log 2>&1; rc=$?
echo "fetch rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- python3 $R/bench.py $ARGS > $OUT/pmc_write.log 2>&1; rc=$?
echo "write rc=$rc"; [ $rc -eq 0 ] || exit $rc
cd $R && python tools/pmc_traffic.py $OUT > $OUT/traffic.log 2>&1; cat $OUT/traffic.log
