#!/bin/bash
# r05n: ECORR LDS-DMA staging (per-chain and shared chunks), late weights, 4-wave workgroups --
# A/B of the ecorr / ecorr_white lines against the round's committed kernel (ecold), the register
# per-chain path (pc0) and 4-wave workgroups (ec4).
set -u
out=gpurun_out/${TAG:-r05n}; mkdir -p $out
export OPENBLAS_NUM_THREADS=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_ecorr.py tests/test_gpu_white.py -m gpu -q --timeout 120 --timeout-method thread -rf > $out/pytest.txt 2>&1
rc=$?; tail -3 $out/pytest.txt; [ $rc -eq 0 ] || exit $rc
for v in ${TEST_VARS:-}; do
  GS_LIB_PATH=$PWD/pulsar_timing_gibbsspec_amd/libpulsar_gibbs_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_ecorr.py tests/test_gpu_white.py -m gpu -q --timeout 120 --timeout-method thread -rf > $out/pytest_$v.txt 2>&1
  rc=$?; echo "tests with $v:"; tail -2 $out/pytest_$v.txt; [ $rc -eq 0 ] || exit $rc
done
for v in ${VARS:-default ecold ec4 ec4m3 default ecold ec4 ec4m3}; do
  if [ "$v" = default ]; then unset GS_LIB_PATH; else export GS_LIB_PATH=$PWD/pulsar_timing_gibbsspec_amd/libpulsar_gibbs_$v.so; fi
  timeout -k 10 300 python bench.py --no-cpu-baseline --pta none --config5 0 --indep 0 --steps 3 --warmup 2 --ecorr-steps 40 > $out/ab_$v.log 2>$out/ab_$v.err || { echo "FAIL $v"; tail -5 $out/ab_$v.err; exit 3; }
  python -c "
import json;d=json.loads(open('$out/ab_$v.log').read().strip().splitlines()[-1]);s=d['secondary']
print('$v', ' '.join('%s %.4e ms/step %.4f kernel %.4f' % (k, v['value'], v['ms_per_step'], v['roofline']['kernel_avg_ms']) for k,v in s.items()))"
done
