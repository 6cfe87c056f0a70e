set -u
mkdir -p gpurun_out/fx
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_indep.py tests/test_gpu_nf.py tests/test_gpu_grid_pta.py tests/test_gpu_pta_mh.py tests/test_gpu_parity.py > gpurun_out/fx/tests.txt 2>&1 || { tail -30 gpurun_out/fx/tests.txt; exit 1; }
tail -2 gpurun_out/fx/tests.txt
for L in default old default old; do
  if [ $L = default ]; then unset GS_LIB_PATH; else export GS_LIB_PATH=$PWD/pulsar_timing_gibbsspec_amd/libpulsar_gibbs_$L.so; fi
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 3 --warmup 1 --config5 0 --ecorr 0 --pta curn,curn_red --pta-ess-sweeps 0 --ess-sweeps 100 --cpu-ess 0 --indep-steps 500 > gpurun_out/fx/b_$L.json 2> gpurun_out/fx/b_$L.err || exit 1
  python -c "
import json; d=json.load(open('gpurun_out/fx/b_$L.json'))
s=d['secondary']; print('$L', 'indep %.4e' % s['indep']['value'], 'indep_ms %.3f' % s['indep']['roofline']['kernel_avg_ms'], {k: ('%.4e' % s[k]['value'], round(s[k]['kernels']['k_bdraw']['kernel_avg_ms'],4)) for k in ('curn','curn_red')})"
done
