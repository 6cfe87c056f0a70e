#!/bin/bash
# r03k: balanced k_bdraw_tiled (contiguous item ranges over the resident workgroups): PTA parity,
# then the PTA lines, balanced (default) vs the 4-group loop (nobal), two passes each.
set -u
mkdir -p gpurun_out/r03k
export OPENBLAS_NUM_THREADS=1
timeout -k 10 500 python -u -m pytest tests/test_gpu_grid_pta.py tests/test_gpu_ks_pta.py -m gpu -x -q \
  --timeout 120 --timeout-method thread > gpurun_out/r03k/pytest.txt 2>&1
rc=$?; tail -3 gpurun_out/r03k/pytest.txt; [ $rc -eq 0 ] || exit $rc
LIBS="default nobal default nobal" PTA=curn_red,curn bash tools/gpu_ab_pta.sh
