#!/bin/bash
# One --pmc pass of <= 8 SQ counters over a python command; per-dispatch means for every kernel
# whose name contains one of KERNELS (space-separated substrings).
#   TAG=x KERNELS="k_rho_red_cert16 k_rho_red_cert(" bash tools/gpu_pmc_kernel.sh tools/ab_red_grid.py 2048 10
set -u
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/pmc_k${TAG:-}
mkdir -p $OUT
export OPENBLAS_NUM_THREADS=1
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 150 rocprofv3 --pmc ${SQ_COUNTERS:-SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU} --output-format csv -d $OUT -o run -- python3 $R/"$@" > $OUT/pmc.log 2>&1; rc=$?
echo "pmc rc=$rc"; tail -2 $OUT/pmc.log
cd $R && python3 - "$OUT" "${KERNELS:-k_}" <<'PY'
import csv, glob, os, sys, collections
d, ks = sys.argv[1], sys.argv[2].split()
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
    for row in csv.DictReader(open(f)):
        name = row.get("Kernel_Name", "")
        for k in ks:
            if k in name:
                acc[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
for k, cs in acc.items():
    print(k)
    for c, v in sorted(cs.items()):
        print("  ", c, len(v), "mean %.4g" % (sum(v) / len(v)))
PY
