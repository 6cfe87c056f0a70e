#!/bin/bash
# r05r: (1) GPU clock under the headline's load (GRBM_GUI_ACTIVE with the kernel trace);
# (2) one FETCH_SIZE pass over configs[4] only (k_white_syrk stages by LDS-DMA since r05k) -- r05q's
# FETCH_SIZE pass over the ECORR lines died in the host (SIGSEGV inside the launch after the first
# LDS-DMA k_ecorr_prefix dispatch); (3) the per-chain ECORR kernel at 3 waves/SIMD (ecpc3) A/B.
set -u
R=$GRAFT_REPO_ROOT
out=$R/gpurun_out/r05r; mkdir -p $out
export OPENBLAS_NUM_THREADS=1
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 150 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace --output-format csv -d $out/grbm -o run -- python3 $R/bench.py --no-cpu-baseline --pta none --config5 0 --indep 0 --ecorr 0 --steps 5 --warmup 2 > $out/grbm.log 2>&1; rc=$?
echo "grbm rc=$rc"; [ $rc -eq 0 ] || exit $rc
cd $R && python3 - <<'PY'
import csv, glob, collections, json
dur = {}
for f in glob.glob("gpurun_out/r05r/grbm/**/*kernel_trace.csv", recursive=True):
    for row in csv.DictReader(open(f)):
        dur[int(row["Dispatch_Id"])] = (row["Kernel_Name"], int(row["End_Timestamp"]) - int(row["Start_Timestamp"]))
clk = collections.defaultdict(list)
for f in glob.glob("gpurun_out/r05r/grbm/**/*counter_collection.csv", recursive=True):
    for row in csv.DictReader(open(f)):
        d = dur.get(int(row["Dispatch_Id"]))
        if d and d[1] > 50000:
            clk[(d[0][:60], row["Counter_Name"])].append((float(row["Counter_Value"]), d[1]))
res = {}
for (k, cn), v in clk.items():
    res.setdefault(k, {})[cn] = {"n": len(v), "counts_per_ns": sum(a for a, _ in v) / sum(b for _, b in v),
                                 "ms_mean": sum(b for _, b in v) / len(v) / 1e6}
json.dump(res, open("gpurun_out/r05r/clock.json", "w"), indent=1)
for k, v in res.items():
    print("clock", k, v)
PY
cd /tmp
timeout -s KILL 170 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $out/syrk_fetch -o run -- python3 $R/bench.py --no-cpu-baseline --pta none --indep 0 --ecorr 0 --steps 2 --warmup 1 --c5-steps 2 > $out/syrk_fetch.log 2>&1; rc=$?
echo "syrk fetch rc=$rc"
cd $R
for v in default ecpc3 default ecpc3; do
  if [ "$v" = default ]; then unset GS_LIB_PATH; else export GS_LIB_PATH=$PWD/pulsar_timing_gibbsspec_amd/libpulsar_gibbs_$v.so; fi
  timeout -k 10 300 python bench.py --no-cpu-baseline --pta none --config5 0 --indep 0 --steps 3 --warmup 2 --ecorr-steps 40 > $out/ab_$v.log 2>$out/ab_$v.err || { echo "FAIL $v"; tail -5 $out/ab_$v.err; exit 3; }
  python -c "
import json;d=json.loads(open('$out/ab_$v.log').read().strip().splitlines()[-1]);s=d['secondary']
print('$v', ' '.join('%s %.4e ms/step %.4f kernel %.4f' % (k, v['value'], v['ms_per_step'], v['roofline']['kernel_avg_ms']) for k,v in s.items()))"
done
