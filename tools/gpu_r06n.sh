#!/bin/bash
# Round 6: k_sweep_pair with both chains' solves interleaved -- bit identity (pair tests), then A/B
# against the sequential solves (libpulsar_gibbs_ilv0.so).
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r06n}
mkdir -p $O
export OPENBLAS_NUM_THREADS=1
cd $R
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py \
  -k "two_chains or handoff or non_pd or cost_model" > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
TAG=${TAG:-r06n} LIBS="${AB_LIBS:-default ilv0}" REPS=3 bash tools/gpu_ab_pair.sh
