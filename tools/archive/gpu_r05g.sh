#!/bin/bash
# r05g: PMC traffic + SQ counters of k_hyper_mh (curn_plred line) and k_white_syrk (configs[4])
set -u
export TESTS=0 SMOKE=0 BENCH=0
PMC="k_hyper_mh k_bdraw_tiled k_rho_curn_fast" PMC_ARGS="--no-cpu-baseline --pta curn_plred --indep 0 --ecorr 0 --config5 0 --host-stream 0 --steps 3 --warmup 1 --ess-sweeps 100 --pta-steps 5 --pta-ess-sweeps 0" bash tools/gpu_full.sh r05g_hyper || exit $?
PMC="k_white_syrk" PMC_ARGS="--no-cpu-baseline --pta none --indep 0 --ecorr 0 --config5 1 --host-stream 0 --steps 3 --warmup 1 --ess-sweeps 100 --c5-steps 2" bash tools/gpu_full.sh r05g_syrk
