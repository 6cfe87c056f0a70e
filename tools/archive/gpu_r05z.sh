#!/bin/bash
# r05z: per-wave ECORR DMA with 3 buffers (chunk i + 2 in flight; default) vs 2 (nb2), each with the
# incremental Metropolis steps (inc=1) and a full evaluation per step (inc=0); ECORR / white tests first.
set -u
R=$GRAFT_REPO_ROOT
out=$R/gpurun_out/r05z; mkdir -p $out
export OPENBLAS_NUM_THREADS=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_ecorr.py tests/test_gpu_white.py -q --timeout 120 --timeout-method thread -rf > $out/pytest.txt 2>&1
rc=$?; tail -3 $out/pytest.txt; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
for v in default nb2; do
for inc in 1 0; do
  if [ "$v" = default ]; then unset GS_LIB_PATH; else export GS_LIB_PATH=$PWD/pulsar_timing_gibbsspec_amd/libpulsar_gibbs_$v.so; fi
  GS_ECORR_INC=$inc timeout -k 10 300 python bench.py --no-cpu-baseline --pta none --config5 0 --indep 0 --steps 3 --warmup 2 --ecorr-steps 40 > $out/ab.log 2>$out/ab.err || { echo "FAIL $v $inc"; tail -5 $out/ab.err; exit 3; }
  python -c "
import json;d=json.loads(open('$out/ab.log').read().strip().splitlines()[-1]);s=d['secondary']
print('$v inc=$inc', ' '.join('%s %.4e ms/step %.4f kernel %.4f' % (k, v['value'], v['ms_per_step'], v['roofline']['kernel_avg_ms']) for k,v in s.items()))"
done; done; done
