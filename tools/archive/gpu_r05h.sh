#!/bin/bash
# r05h: likelihood-mode logs (gs_log_pos vs libm) on the PTA MH line; parity of the lnl users
set -u
bash tools/gpu_tests.sh r05h tests/test_gpu_pta_mh.py tests/test_gpu_lnlike.py tests/test_gpu_pta_api.py tests/test_gpu_red.py tests/test_gpu_big.py || exit $?
mkdir -p gpurun_out/r05h
LIBS="default lnllibm default lnllibm" STEPS=50 PTA=curn_plred BENCH_ARGS="--pta-ess-sweeps 0 --indep 0 --ecorr 0" bash tools/gpu_ab_lib.sh 2>&1 | tee gpurun_out/r05h/ab_lnl.txt
for v in default lnllibm; do grep -o '"k_hyper_mh": {"kernel_avg_ms": [0-9.]*' gpurun_out/ab_${v}_c4096.log; grep -o '"k_bdraw": {"kernel_avg_ms": [0-9.]*' gpurun_out/ab_${v}_c4096.log; done
