#!/bin/bash
# r05z15: PMC traffic (FETCH_SIZE, WRITE_SIZE in separate passes) of the configs[2] fused sweep
# (k_sweep_freespec_rm, 45 pulsars x 256 chains, 100 sweeps per launch; largest dispatch)
set -u
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/pmc_indep
mkdir -p $OUT
export OPENBLAS_NUM_THREADS=1
ARGS="--no-cpu-baseline --pta none --ecorr 0 --config5 0 --host-stream 0 --steps 2 --warmup 1 --ess-sweeps 100 --indep-steps 300"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 170 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- python3 $R/bench.py $ARGS > $OUT/fetch.log 2>&1; rc=$?
echo "fetch rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 170 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- python3 $R/bench.py $ARGS > $OUT/write.log 2>&1; rc=$?
echo "write rc=$rc"; [ $rc -eq 0 ] || exit $rc
cd $R && python3 - <<'PY'
import csv, collections
for tag in ("pmc_fetch", "pmc_write"):
    rows = list(csv.DictReader(open(f"gpurun_out/pmc_indep/{tag}/run_counter_collection.csv")))
    c = collections.Counter((r["Kernel_Name"][:70], r["Grid_Size"]) for r in rows if "sweep_freespec_rm" in r["Kernel_Name"])
    print(tag, c.most_common(4))
PY
SWEEPS=100 CHAINS=11520 GRID=${GRID:-737280} HEAD_LAUNCHES=0 python tools/pmc_traffic.py $OUT "k_sweep_freespec_rm" $OUT/pmc_traffic_indep.json
