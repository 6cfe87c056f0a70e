#!/bin/bash
# Round 6: WRITE_SIZE of the ECORR step kernel (FETCH_SIZE came from r06c), then LAST the round-5 PMC
# crash command (bench.py's headline + ECORR lines under --pmc FETCH_SIZE) with maps written.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r06d}
mkdir -p $O
export OPENBLAS_NUM_THREADS=1
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/wr -o run -- \
  python3 $R/tools/ecorr_pmc_probe.py $O/wr_maps 4096 > $O/wr.log 2>&1
rc=$?; echo "wr rc=$rc"; tail -2 $O/wr.log
[ $rc -eq 0 ] || exit $rc
GS_MAPS_OUT=$O/maps.txt timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc -o run -- \
  python3 $R/tools/bench_maps.py --no-cpu-baseline --pta none --config5 0 --indep 0 --steps 2 --warmup 1 \
  --ecorr-steps 2 --ess 0 > $O/pmc.json 2> $O/pmc.log
echo "pmc rc=$?"; tail -45 $O/pmc.log
