#!/bin/bash
# r04b: GPU tests touched in round 4 (PTA MH, CURN sum pinning, contraction fixes, 16-lane red grid)
set -u
out=gpurun_out/r04b
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_gpu_pta_mh.py tests/test_gpu_grid_pta.py tests/test_gpu_white.py \
  tests/test_gpu_ecorr.py tests/test_gpu_parity.py tests/test_gpu_red.py tests/test_gpu_ks_pta.py tests/test_gpu_nf.py \
  -q --timeout 120 --timeout-method thread -rf > $out/pytest.txt 2>&1
rc=$?; tail -12 $out/pytest.txt
exit $rc
