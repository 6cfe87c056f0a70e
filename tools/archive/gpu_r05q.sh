#!/bin/bash
# r05q: the ECORR tests on the round-5 ECORR kernel (staging edge cases), then its PMC traffic
# (tools/archive/gpu_pmc_ecorr.sh) and one SQ pass over the same bench command.
set -u
out=gpurun_out/r05q; mkdir -p $out
export OPENBLAS_NUM_THREADS=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_ecorr.py tests/test_gpu_white.py tests/test_kernel_resources.py -q --timeout 120 --timeout-method thread -rf > $out/pytest.txt 2>&1
rc=$?; tail -4 $out/pytest.txt; [ $rc -eq 0 ] || exit $rc
bash tools/archive/gpu_pmc_ecorr.sh || exit $?
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_MISC SQ_WAVES --output-format csv -d $R/gpurun_out/pmc_ecorr/sq -o run -- python3 $R/bench.py --no-cpu-baseline --pta none --config5 0 --indep 0 --steps 3 --warmup 2 --ecorr-steps 2 > $R/$out/sq.log 2>&1; rc=$?
echo "sq rc=$rc"; [ $rc -eq 0 ] || exit $rc
# GPU clock under load: GRBM_GUI_ACTIVE (GPU-busy clock cycles per dispatch) with the kernel trace's
# durations of the same dispatches
timeout -s KILL 150 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace --output-format csv -d $R/gpurun_out/pmc_ecorr/grbm -o run -- python3 $R/bench.py --no-cpu-baseline --pta none --config5 0 --indep 0 --steps 3 --warmup 2 --ecorr-steps 2 > $R/$out/grbm.log 2>&1; rc=$?
echo "grbm rc=$rc"; [ $rc -eq 0 ] || exit $rc
cd $R && python3 - <<'PY'
import csv, glob, collections, json
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob("gpurun_out/pmc_ecorr/sq/**/*counter_collection.csv", recursive=True):
    for row in csv.DictReader(open(f)):
        n = row.get("Kernel_Name", "")
        if "k_ecorr_prefix<5, true" in n and int(row.get("Grid_Size", 0)) == 4096 * 64:
            acc[n][row["Counter_Name"]].append(float(row["Counter_Value"]))
out = {n: {c: sum(v) / len(v) for c, v in cs.items()} for n, cs in acc.items()}
json.dump(out, open("gpurun_out/r05q/sq.json", "w"), indent=1)
for n, cs in out.items():
    print(n[:60], {c: round(v) for c, v in cs.items()})
# clock: GRBM_GUI_ACTIVE / kernel-trace duration, per dispatch, for the big kernels
dur = {}
for f in glob.glob("gpurun_out/pmc_ecorr/grbm/**/*kernel_trace.csv", recursive=True):
    for row in csv.DictReader(open(f)):
        dur[int(row["Dispatch_Id"])] = (row["Kernel_Name"], int(row["End_Timestamp"]) - int(row["Start_Timestamp"]))
clk = collections.defaultdict(list)
for f in glob.glob("gpurun_out/pmc_ecorr/grbm/**/*counter_collection.csv", recursive=True):
    for row in csv.DictReader(open(f)):
        if row["Counter_Name"] != "GRBM_GUI_ACTIVE":
            continue
        d = dur.get(int(row["Dispatch_Id"]))
        if d and d[1] > 50000:
            clk[d[0][:70]].append((float(row["Counter_Value"]) / d[1], d[1] / 1e6))
res = {k: {"n": len(v), "ghz_mean": sum(x for x, _ in v) / len(v), "ms_mean": sum(y for _, y in v) / len(v)} for k, v in clk.items()}
json.dump(res, open("gpurun_out/r05q/clock.json", "w"), indent=1)
for k, v in res.items():
    print("clock", k, v)
PY
# A/B: the per-chain kernel at 3 waves/SIMD (ecpc3: 168 VGPRs, 54 spilled) against the default (240, 2/SIMD)
cd $R
for v in default ecpc3 default ecpc3; do
  if [ "$v" = default ]; then unset GS_LIB_PATH; else export GS_LIB_PATH=$PWD/pulsar_timing_gibbsspec_amd/libpulsar_gibbs_$v.so; fi
  timeout -k 10 300 python bench.py --no-cpu-baseline --pta none --config5 0 --indep 0 --steps 3 --warmup 2 --ecorr-steps 40 > $out/ab_$v.log 2>$out/ab_$v.err || { echo "FAIL $v"; tail -5 $out/ab_$v.err; exit 3; }
  python -c "
import json;d=json.loads(open('$out/ab_$v.log').read().strip().splitlines()[-1]);s=d['secondary']
print('$v', ' '.join('%s %.4e ms/step %.4f kernel %.4f' % (k, v['value'], v['ms_per_step'], v['roofline']['kernel_avg_ms']) for k,v in s.items()))"
done
