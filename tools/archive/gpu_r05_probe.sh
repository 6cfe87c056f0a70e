#!/bin/bash
# r05: DPP-from-disabled-lane probe, cost attribution of the sweep's pre-factorisation phases,
# XCD-major k_bdraw_tiled ranges A/B
set -u
mkdir -p gpurun_out/r05b
timeout -k 10 60 ./tools/probe/dpp_exec_probe > gpurun_out/r05b/dpp_exec_probe.txt 2>&1; cat gpurun_out/r05b/dpp_exec_probe.txt
LIBS="default pnophil pnolog pnonorm default" STEPS=300 bash tools/gpu_ab_lib.sh 2>&1 | tee gpurun_out/r05b/ab.txt || exit 3
LIBS="default bxcd0 default bxcd0" STEPS=100 PTA=curn,curn_plred BENCH_ARGS="--pta-ess-sweeps 0" bash tools/gpu_ab_lib.sh 2>&1 | tee gpurun_out/r05b/ab_pta.txt
