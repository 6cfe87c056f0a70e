#!/bin/bash
# r03j: hybrid tiled layout (row-major fixed block for nm > 16): parity (PTA, configs[2], single
# pulsar), then headline + indep lines and the PTA lines with / without the tiled PTA draws.
set -u
mkdir -p gpurun_out/r03j
export OPENBLAS_NUM_THREADS=1
timeout -k 10 500 python -u -m pytest tests/test_gpu_grid_pta.py tests/test_gpu_indep.py tests/test_gpu_parity.py tests/test_gpu_nf.py \
  -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03j/pytest.txt 2>&1
rc=$?; tail -3 gpurun_out/r03j/pytest.txt; [ $rc -eq 0 ] || exit $rc
LIBS=default bash tools/gpu_ab_lib.sh || exit 3
for t in 1 0 1 0; do
  GS_PTA_TILED=$t PTA=curn_red,curn bash tools/gpu_ab_pta.sh && cp gpurun_out/abp_default.json gpurun_out/r03j/abp_tiled$t.json || exit 3
done
