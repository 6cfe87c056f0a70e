#!/bin/bash
# r03f: rcp-DPP probe (expected to fail: documents the hardware result), parity of the tiled-model
# sweep + MFMA-neg tile core, then headline A/B (untiled / noneg / minw3 / default) and the CURN line.
set -u
mkdir -p gpurun_out/r03f
export OPENBLAS_NUM_THREADS=1
timeout -k 10 60 ./tools/probe/rcpdpp_probe > gpurun_out/r03f/rcpdpp_probe.txt; cat gpurun_out/r03f/rcpdpp_probe.txt
PT="tests/test_gpu_parity.py tests/test_gpu_nf.py tests/test_gpu_grid_pta.py tests/test_gpu_big.py"
GS_LIB_PATH=$PWD/pulsar_timing_gibbsspec_amd/libpulsar_gibbs_untiled.so timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py \
  -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03f/pytest_untiled.txt 2>&1
echo "untiled lib parity rc=$?"; tail -2 gpurun_out/r03f/pytest_untiled.txt
timeout -k 10 400 python -u -m pytest $PT -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03f/pytest.txt 2>&1
rc=$?; tail -3 gpurun_out/r03f/pytest.txt; [ $rc -eq 0 ] || exit $rc
LIBS="${LIBS:-untiled noneg minw3 default untiled noneg minw3 default}" bash tools/gpu_ab_lib.sh || exit 3
LIBS="${PLIBS:-default}" PTA=curn bash tools/gpu_ab_pta.sh
