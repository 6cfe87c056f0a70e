#!/bin/bash
# Round 6: whole GPU suite on the current library, then a headline A/B against variant libraries
# (AB_LIBS, built with csrc/Makefile variant-one).
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r06q}
mkdir -p $O
export OPENBLAS_NUM_THREADS=1
cd $R
export GS_PARITY_REPORT=$O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -rf > $O/pytest.txt 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.txt; [ $rc -eq 0 ] || exit $rc
TAG=${TAG:-r06q} LIBS="${AB_LIBS:-default}" REPS=${REPS:-3} bash tools/gpu_ab_pair.sh
