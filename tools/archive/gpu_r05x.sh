#!/bin/bash
# r05x: SQ counters of the configs[4] SYRK (k_white_syrk<14>, LDS-DMA staging since r05k)
set -u
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r05x
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU"
TAG=sy KERNELS="k_white_syrk<14>" SQ_COUNTERS="$SQ" bash tools/gpu_pmc_kernel.sh bench.py --no-cpu-baseline --pta none --indep 0 --ecorr 0 --steps 2 --warmup 1 --c5-steps 2 --ess-sweeps 100 > $R/gpurun_out/r05x/sy.txt 2>&1; rc=$?
cat $R/gpurun_out/r05x/sy.txt | grep -v "^W2026"; [ $rc -eq 0 ] || exit $rc
SQ2="SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM SQ_INSTS_SALU"
TAG=sy2 KERNELS="k_white_syrk<14>" SQ_COUNTERS="$SQ2" bash tools/gpu_pmc_kernel.sh bench.py --no-cpu-baseline --pta none --indep 0 --ecorr 0 --steps 2 --warmup 1 --c5-steps 2 --ess-sweeps 100 > $R/gpurun_out/r05x/sy2.txt 2>&1; rc=$?
cat $R/gpurun_out/r05x/sy2.txt | grep -v "^W2026"; exit $rc
