#!/bin/bash
# PMC traffic (FETCH_SIZE, WRITE_SIZE in separate passes) of the configs[3] CURN + red line's
# kernels: k_rho_red_cert16 (45 pulsars x 30 bins x 2048 chains = 2.76 M rows, 64 per wave: grid
# 10800 x 256 work-items) and k_bdraw_tiled (92160 systems: grid 45 x 128 x 256).
set -u
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/pmc_red
mkdir -p $OUT
export OPENBLAS_NUM_THREADS=1
ARGS="--no-cpu-baseline --pta curn_red --indep 0 --ecorr 0 --config5 0 --host-stream 0 --steps 3 --warmup 1 --ess-sweeps 100 --pta-steps 5 --pta-ess-sweeps 0"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 170 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- python3 $R/bench.py $ARGS > $OUT/fetch.log 2>&1; rc=$?
echo "fetch rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 170 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- python3 $R/bench.py $ARGS > $OUT/write.log 2>&1; rc=$?
echo "write rc=$rc"; [ $rc -eq 0 ] || exit $rc
cd $R && SWEEPS=1 CHAINS=2048 GRID=2764800 HEAD_LAUNCHES=6 python tools/pmc_traffic.py $OUT "k_rho_red_cert16" $OUT/pmc_traffic_red.json && \
  SWEEPS=1 CHAINS=92160 GRID=196608 HEAD_LAUNCHES=6 python tools/pmc_traffic.py $OUT "k_bdraw_tiled<60" $OUT/pmc_traffic_red_bdraw.json
