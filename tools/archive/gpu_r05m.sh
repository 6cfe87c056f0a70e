#!/bin/bash
# r05m: PMC traffic of k_bdraw_tiled (CURN line, every chain drawing) with workgroup-order vs XCD-major
# persistent ranges, plus the graph-replay test of the red MH counts
set -u
bash tools/gpu_tests.sh r05m "tests/test_gpu_grid_pta.py::test_graph_replay_equals_eager_sweeps" || exit $?
export TESTS=0 SMOKE=0 BENCH=0
ARGS="--no-cpu-baseline --pta curn --indep 0 --ecorr 0 --config5 0 --host-stream 0 --steps 3 --warmup 1 --ess-sweeps 100 --pta-steps 5 --pta-ess-sweeps 0"
PMC="k_bdraw_tiled" PMC_ARGS="$ARGS" bash tools/gpu_full.sh r05m_wg || exit $?
GS_LIB_PATH=$PWD/pulsar_timing_gibbsspec_amd/libpulsar_gibbs_bxcd1.so PMC="k_bdraw_tiled" PMC_ARGS="$ARGS" bash tools/gpu_full.sh r05m_xcd
