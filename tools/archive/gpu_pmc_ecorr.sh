#!/bin/bash
# PMC traffic (FETCH_SIZE, WRITE_SIZE in separate passes) of the two ECORR likelihood kernels.
set -u
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/pmc_ecorr
mkdir -p $OUT
export OPENBLAS_NUM_THREADS=1
ARGS="--no-cpu-baseline --pta none --config5 0 --steps 10 --warmup 2 --ecorr-steps 2"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- python3 $R/bench.py $ARGS > $OUT/fetch.log 2>&1; rc=$?
echo "fetch rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- python3 $R/bench.py $ARGS > $OUT/write.log 2>&1; rc=$?
echo "write rc=$rc"; [ $rc -eq 0 ] || exit $rc
# both likelihood kernels run in the same passes (bench's ecorr and ecorr_white lines)
cd $R && SWEEPS=1 CHAINS=4096 python tools/pmc_traffic.py $OUT "k_ecorr_prefix<5, true, false>" $OUT/pmc_traffic_ecorr.json \
  && SWEEPS=1 CHAINS=4096 python tools/pmc_traffic.py $OUT "k_ecorr_prefix<5, true, true>" $OUT/pmc_traffic_ecorr_white.json
