#!/bin/bash
# Round 6: the cost model now runs the headline on k_sweep_pair.  Whole GPU suite, then the headline's
# HBM traffic (FETCH_SIZE, WRITE_SIZE passes) and a kernel-trace of the default headline command.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r06m}
mkdir -p $O
export OPENBLAS_NUM_THREADS=1
cd $R
export GS_PARITY_REPORT=$O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -rf > $O/pytest.txt 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 $O/pytest.txt; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
ARGS="--no-cpu-baseline --ess 0 --indep 0 --pta none --ecorr 0 --config5 0 --host-stream 0 --steps 20 --warmup 5"
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 170 rocprofv3 --pmc $C --output-format csv -d $O/$C -o run -- python3 $R/bench.py $ARGS > $O/$C.json 2> $O/$C.log
  rc=$?; echo "$C rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 170 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 $R/bench.py $ARGS \
  > $O/kt_bench.json 2> $O/kt.log
rc=$?; echo "kt rc=$rc"; [ $rc -eq 0 ] || exit $rc
find $O/kt -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats.csv \;
find $O/kt -name "*kernel_trace.csv" -exec rm {} \;
head -3 $O/kernel_stats.csv
