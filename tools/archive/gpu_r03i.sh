#!/bin/bash
# r03i: tiled model copies for the PTA b draws (gs_model_tile + gs_bdraw_tiled): PTA parity and KS
# tests, then the CURN / CURN+red lines with and without them (GS_PTA_TILED=0).
set -u
mkdir -p gpurun_out/r03i
export OPENBLAS_NUM_THREADS=1
timeout -k 10 500 python -u -m pytest tests/test_gpu_grid_pta.py tests/test_gpu_ks_pta.py tests/test_gpu_dist.py -m gpu -x -q \
  --timeout 120 --timeout-method thread > gpurun_out/r03i/pytest.txt 2>&1
rc=$?; tail -3 gpurun_out/r03i/pytest.txt; [ $rc -eq 0 ] || exit $rc
for t in 1 0 1 0; do
  GS_PTA_TILED=$t PTA=curn_red,curn bash tools/gpu_ab_pta.sh && cp gpurun_out/abp_default.json gpurun_out/r03i/abp_tiled$t.json || exit 3
done
