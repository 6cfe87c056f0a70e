#!/bin/bash
# r05z11: the ECORR Metropolis step fused into one launch (gs_ecorr_mh_step) -- ECORR / white tests,
# then an interleaved A/B of the ecorr lines with the fused step (default) and the two-launch step
# (GS_ECORR_FUSE=0)
set -u
R=$GRAFT_REPO_ROOT
out=$R/gpurun_out/r05z11; mkdir -p $out
export OPENBLAS_NUM_THREADS=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_ecorr.py tests/test_gpu_white.py -q --timeout 120 --timeout-method thread -rf > $out/pytest.txt 2>&1
rc=$?; tail -4 $out/pytest.txt; [ $rc -eq 0 ] || exit $rc
GS_ECORR_FUSE=0 timeout -k 10 400 python -u -m pytest tests/test_gpu_ecorr.py -q --timeout 120 --timeout-method thread -rf -k "incremental or matches_reference" > $out/pytest_nofuse.txt 2>&1
rc=$?; tail -2 $out/pytest_nofuse.txt; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
for v in 1 0; do
  GS_ECORR_FUSE=$v timeout -k 10 300 python bench.py --no-cpu-baseline --pta none --config5 0 --indep 0 --steps 3 --warmup 2 --ecorr-steps 40 > $out/ab.log 2>$out/ab.err || { echo "FAIL $v"; tail -5 $out/ab.err; exit 3; }
  python -c "
import json;d=json.loads(open('$out/ab.log').read().strip().splitlines()[-1]);s=d['secondary']
print('fuse=$v', ' '.join('%s %.4e ms/step %.4f' % (k, v['value'], v['ms_per_step']) for k,v in s.items()))"
done; done
