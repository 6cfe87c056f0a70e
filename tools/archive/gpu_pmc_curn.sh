#!/bin/bash
# PMC traffic (FETCH_SIZE, WRITE_SIZE in separate passes) of k_bdraw_tiled in the configs[3] CURN
# line (45 pulsars x 2048 chains = 92160 systems, one wavefront each, 4 chain groups of 4 waves per
# workgroup; round 4: one persistent round of 768 workgroups x 256 work-items on 256 CUs).
set -u
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/pmc_curn
mkdir -p $OUT
export OPENBLAS_NUM_THREADS=1
ARGS="--no-cpu-baseline --pta curn --indep 0 --ecorr 0 --config5 0 --host-stream 0 --steps 3 --warmup 1 --ess-sweeps 100 --pta-steps 5 --pta-ess-sweeps 0"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- python3 $R/bench.py $ARGS > $OUT/fetch.log 2>&1; rc=$?
echo "fetch rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- python3 $R/bench.py $ARGS > $OUT/write.log 2>&1; rc=$?
echo "write rc=$rc"; [ $rc -eq 0 ] || exit $rc
cd $R && SWEEPS=1 CHAINS=92160 GRID=${GRID:-196608} HEAD_LAUNCHES=6 python tools/pmc_traffic.py $OUT "k_bdraw_tiled<60" $OUT/pmc_traffic_curn.json
