#!/bin/bash
# SQ issue/stall counters of the headline sweep kernel: one --pmc pass of <= 8 SQ counters
# (MI355X_MICROARCH.md: WAIT_ANY + WAIT_INST_ANY + ACTIVE_INST_ANY ~ WAVE_CYCLES, quad-cycles).
set -u
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/pmc_sq${TAG:-}
mkdir -p $OUT
export OPENBLAS_NUM_THREADS=1
ARGS="--no-cpu-baseline --indep 0 --pta none --ecorr 0 --config5 0 --host-stream 0 --steps 200 --warmup 10 ${BENCH_ARGS:-}"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc ${SQ_COUNTERS:-SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_MFMA SQ_BUSY_CYCLES} --output-format csv -d $OUT -o run -- python3 $R/bench.py $ARGS > $OUT/pmc.log 2>&1; rc=$?
echo "pmc rc=$rc"; tail -3 $OUT/pmc.log
cd $R && python3 - "$OUT" <<'PY'
import csv, glob, os, sys, collections
d = sys.argv[1]
acc = collections.defaultdict(list)
for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
    for row in csv.DictReader(open(f)):
        if "k_sweep_freespec" in row.get("Kernel_Name", ""):
            acc[row["Counter_Name"]].append(float(row["Counter_Value"]))
for k, v in sorted(acc.items()):
    print(k, len(v), "per-dispatch mean %.4g" % (sum(v[1:]) / max(1, len(v) - 1) if len(v) > 1 else v[0]))
PY
