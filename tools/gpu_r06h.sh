#!/bin/bash
# Round 6: the headline kernel's HBM traffic re-measured on this round's library (FETCH_SIZE and
# WRITE_SIZE in separate passes over the headline-only bench command, 5 warm-up + 20 timed launches).
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r06h}
mkdir -p $O
export OPENBLAS_NUM_THREADS=1
cd /tmp && export TMPDIR=/tmp
ARGS="--no-cpu-baseline --ess 0 --indep 0 --pta none --ecorr 0 --config5 0 --host-stream 0 --steps 20 --warmup 5"
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 170 rocprofv3 --pmc $C --output-format csv -d $O/$C -o run -- python3 $R/bench.py $ARGS > $O/$C.json 2> $O/$C.log
  rc=$?; echo "$C rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
