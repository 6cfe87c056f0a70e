#!/bin/bash
# r05z13: PMC traffic (FETCH_SIZE, WRITE_SIZE in separate passes) of k_bdraw_tiled with the lnL output
# in the configs[3] curn_plred line (45 x 2048 systems; the largest dispatch = every chain drawing,
# the bench's HIP-event launch)
set -u
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/pmc_plred
mkdir -p $OUT
export OPENBLAS_NUM_THREADS=1
ARGS="--no-cpu-baseline --pta curn_plred --indep 0 --ecorr 0 --config5 0 --host-stream 0 --steps 3 --warmup 1 --ess-sweeps 100 --pta-steps 5 --pta-ess-sweeps 0"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 170 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- python3 $R/bench.py $ARGS > $OUT/fetch.log 2>&1; rc=$?
echo "fetch rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 170 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- python3 $R/bench.py $ARGS > $OUT/write.log 2>&1; rc=$?
echo "write rc=$rc"; [ $rc -eq 0 ] || exit $rc
cd $R && SWEEPS=1 CHAINS=92160 GRID=${GRID:-196608} HEAD_LAUNCHES=0 python tools/pmc_traffic.py $OUT "k_bdraw_tiled<60" $OUT/pmc_traffic_plred_bdraw.json
