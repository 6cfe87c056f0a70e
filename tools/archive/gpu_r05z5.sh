#!/bin/bash
# r05z5: cost attribution of the incremental ECORR step kernel: without the stored-state load
# (noload, acc from Ap) and without the proposal-state store (nostore) -- timing only (wrong draws)
set -u
R=$GRAFT_REPO_ROOT
out=$R/gpurun_out/r05z5; mkdir -p $out
export OPENBLAS_NUM_THREADS=1
for rep in 1 2; do
for v in default noload nostore; do
  if [ "$v" = default ]; then unset GS_LIB_PATH; else export GS_LIB_PATH=$PWD/pulsar_timing_gibbsspec_amd/libpulsar_gibbs_$v.so; fi
  timeout -k 10 300 python bench.py --no-cpu-baseline --pta none --config5 0 --indep 0 --steps 3 --warmup 2 --ecorr-steps 10 > $out/ab.log 2>$out/ab.err || { echo "FAIL $v"; tail -5 $out/ab.err; exit 3; }
  python -c "
import json;d=json.loads(open('$out/ab.log').read().strip().splitlines()[-1]);s=d['secondary']
print('$v', ' '.join('%s full %.4f step %.4f' % (k, v['roofline']['kernel_avg_ms'], v['step_roofline']['kernel_avg_ms']) for k,v in s.items()))"
done; done
