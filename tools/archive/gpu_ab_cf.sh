#!/bin/bash
# CURN product kernel A/B (default vs libpulsar_gibbs_old.so) on the CURN + red line, after its tests
set -u
mkdir -p gpurun_out/cf
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_grid_pta.py > gpurun_out/cf/tests.txt 2>&1 || { tail -30 gpurun_out/cf/tests.txt; exit 1; }
tail -2 gpurun_out/cf/tests.txt
ALT=${ALT:-old}
for L in default $ALT default $ALT; do
  if [ $L = default ]; then unset GS_LIB_PATH; else export GS_LIB_PATH=$PWD/pulsar_timing_gibbsspec_amd/libpulsar_gibbs_$L.so; fi
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 3 --warmup 1 --indep 0 --config5 0 --ecorr 0 --pta curn_red --pta-ess-sweeps 0 --ess-sweeps 100 --cpu-ess 0 > gpurun_out/cf/b_$L.json 2> gpurun_out/cf/b_$L.err || exit 1
  python -c "
import json; d=json.load(open('gpurun_out/cf/b_$L.json'))
s=d['secondary']['curn_red']; print('$L', '%.4e' % s['value'], round(s['ms_per_step'],4), {k: round(v['kernel_avg_ms'],4) for k,v in s['kernels'].items()})"
done
