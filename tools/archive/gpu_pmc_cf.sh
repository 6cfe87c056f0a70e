#!/bin/bash
# SQ counters of the CURN + red line's kernels (one --pmc pass, the default 8 SQ counters)
set -u
TAG=${TAG:-cf} KERNELS="k_rho_curn_fast k_bdraw_tiled k_rho_red_cert16 k_hyper_mh" timeout -k 10 200 bash tools/gpu_pmc_kernel.sh bench.py --no-cpu-baseline --steps 3 --warmup 1 --indep 0 --config5 0 --ecorr 0 --pta curn_red,curn_plred --pta-ess-sweeps 0 --ess-sweeps 100 --cpu-ess 0
