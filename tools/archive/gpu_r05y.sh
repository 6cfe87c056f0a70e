#!/bin/bash
# r05y: incremental ECORR Metropolis steps (gs_ecorr_lnl_state) -- the ECORR / white GPU tests, then
# an interleaved A/B of the ecorr lines with the incremental steps (default) and a full evaluation
# per step (GS_ECORR_INC=0).
set -u
R=$GRAFT_REPO_ROOT
out=$R/gpurun_out/r05y; mkdir -p $out
export OPENBLAS_NUM_THREADS=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_ecorr.py tests/test_gpu_white.py -q --timeout 120 --timeout-method thread -rf > $out/pytest.txt 2>&1
rc=$?; tail -6 $out/pytest.txt; [ $rc -eq 0 ] || exit $rc
for v in 1 0 1 0; do
  GS_ECORR_INC=$v timeout -k 10 300 python bench.py --no-cpu-baseline --pta none --config5 0 --indep 0 --steps 3 --warmup 2 --ecorr-steps 40 > $out/ab_$v.log 2>$out/ab_$v.err || { echo "FAIL $v"; tail -5 $out/ab_$v.err; exit 3; }
  python -c "
import json;d=json.loads(open('$out/ab_$v.log').read().strip().splitlines()[-1]);s=d['secondary']
print('inc=$v', ' '.join('%s %.4e ms/step %.4f kernel %.4f ess %.4g' % (k, v['value'], v['ms_per_step'], v['roofline']['kernel_avg_ms'], v['ess']['per_chain_sweep_min_bin']) for k,v in s.items()))"
done
