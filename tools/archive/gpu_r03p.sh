#!/bin/bash
# r03p: the extended tiled-vs-row-major b-draw test (nm <= 16 fixed block in tiles, NF = 40)
set -u
mkdir -p gpurun_out/r03p
export OPENBLAS_NUM_THREADS=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_grid_pta.py -k "tiled" -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r03p/pytest.txt 2>&1; rc=$?; tail -3 gpurun_out/r03p/pytest.txt; exit $rc
