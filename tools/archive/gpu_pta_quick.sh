mkdir -p gpurun_out/lnl
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_lnlike.py tests/test_gpu_pta_mh.py tests/test_gpu_grid_pta.py tests/test_gpu_dist.py > gpurun_out/lnl/pytest.txt 2>&1 || { tail -20 gpurun_out/lnl/pytest.txt; exit 1; }
tail -2 gpurun_out/lnl/pytest.txt
timeout -k 10 400 python -u bench.py --no-cpu-baseline --steps 3 --warmup 1 --indep 0 --config5 0 --ecorr 0 --pta curn,curn_plred,curn_red --cpu-ess 0 > gpurun_out/lnl/bench.json 2> gpurun_out/lnl/bench.err || { tail -5 gpurun_out/lnl/bench.err; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/lnl/bench.json'))
for k,v in d['secondary'].items():
    print(k, '%.4g'%v['value'], 'ms/step %.3f'%v['ms_per_step'], {kk: round(vv['kernel_avg_ms'],3) for kk,vv in v.get('kernels',{}).items()}, v.get('kernels',{}).get('k_rho_red_cert16',{}).get('f64_redo_rows_frac'))
"
