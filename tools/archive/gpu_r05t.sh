#!/bin/bash
# r05t: the GPU's shader clock while the headline kernel runs back to back (rocm-smi polled every
# 0.5 s during a 4000-launch bench run), against idle.
set -u
R=$GRAFT_REPO_ROOT
out=$R/gpurun_out/r05t; mkdir -p $out
export OPENBLAS_NUM_THREADS=1
rocm-smi --showclocks --showpower --showtemp > $out/smi_idle.txt 2>&1
timeout -k 10 150 python bench.py --no-cpu-baseline --pta none --config5 0 --indep 0 --ecorr 0 --steps 4000 --warmup 5 --ess-sweeps 200 > $out/long.json 2> $out/long.err &
pid=$!
for i in $(seq 1 40); do
  echo "=== $i $(date +%s.%N)" >> $out/smi_load.txt
  rocm-smi --showclocks --showpower --showtemp >> $out/smi_load.txt 2>&1
  sleep 0.5
done
wait $pid; rc=$?
echo "bench rc=$rc"
grep -h "sclk\|Power\|Temperature (Sensor junction)" $out/smi_load.txt | sort | uniq -c | sort -rn | head -20
python -c "import json;d=json.load(open('$out/long.json'));print('kernel ms', d['roofline']['kernel_avg_ms'], 'ms/step', d['ms_per_step'])"
exit $rc
