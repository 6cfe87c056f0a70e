#!/bin/bash
# PMC HBM traffic (FETCH_SIZE and WRITE_SIZE, separate passes) + one SQ pass of a bench.py command,
# averaged per dispatch for each kernel whose name contains one of KERNELS.
#   TAG=hyper KERNELS="k_hyper_mh k_bdraw_tiled" BENCH_ARGS="--pta curn_plred ..." bash tools/gpu_pmc_traffic.sh
set -u
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/pmc_${TAG:-x}
mkdir -p $OUT
export OPENBLAS_NUM_THREADS=1
cd /tmp && export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE "${SQ:-SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES}"; do
  tag=$(echo $C | cut -d' ' -f1)
  timeout -s KILL 170 rocprofv3 --pmc $C --output-format csv -d $OUT/$tag -o run -- python3 $R/bench.py $BENCH_ARGS > $OUT/$tag.log 2>&1; rc=$?
  echo "$tag rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
cd $R && python3 - "$OUT" "${KERNELS}" <<'PY'
import csv, glob, json, os, sys, collections
d, ks = sys.argv[1], sys.argv[2].split()
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
    for row in csv.DictReader(open(f)):
        name = row.get("Kernel_Name", "")
        for k in ks:
            if k in name:
                acc[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
out = {}
for k, cs in acc.items():
    m = {c: sum(v) / len(v) for c, v in cs.items()}
    m["dispatches"] = {c: len(v) for c, v in cs.items()}
    if "FETCH_SIZE" in m and "WRITE_SIZE" in m:
        # KiB; FETCH_SIZE x 2 on gfx950 for streaming reads (MI355X_MICROARCH.md, tools/pmc_traffic.py)
        m["traffic_bytes_per_launch"] = (2 * m["FETCH_SIZE"] + m["WRITE_SIZE"]) * 1024
    out[k] = m
    print(k, {c: (round(v, 1) if isinstance(v, float) else v) for c, v in m.items() if c != "dispatches"})
json.dump(out, open(os.path.join(d, "pmc_summary.json"), "w"), indent=1)
PY
