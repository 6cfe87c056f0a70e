#!/bin/bash
# r05z2: the incremental ECORR step at 3 waves/SIMD (inc3: 168 VGPRs, 59 spilled) vs 2 (default, 230)
set -u
R=$GRAFT_REPO_ROOT
out=$R/gpurun_out/r05z2; mkdir -p $out
export OPENBLAS_NUM_THREADS=1
for rep in 1 2; do
for v in default inc3; do
  if [ "$v" = default ]; then unset GS_LIB_PATH; else export GS_LIB_PATH=$PWD/pulsar_timing_gibbsspec_amd/libpulsar_gibbs_$v.so; fi
  timeout -k 10 300 python bench.py --no-cpu-baseline --pta none --config5 0 --indep 0 --steps 3 --warmup 2 --ecorr-steps 40 > $out/ab.log 2>$out/ab.err || { echo "FAIL $v"; tail -5 $out/ab.err; exit 3; }
  python -c "
import json;d=json.loads(open('$out/ab.log').read().strip().splitlines()[-1]);s=d['secondary']
print('$v', ' '.join('%s %.4e ms/step %.4f kernel %.4f' % (k, v['value'], v['ms_per_step'], v['roofline']['kernel_avg_ms']) for k,v in s.items()))"
done; done
