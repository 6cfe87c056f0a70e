#!/bin/bash
# Round-end check on one GPU: the whole GPU suite, then smoke() (the driver's two GPU tiers).
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-final}
mkdir -p $O
export OPENBLAS_NUM_THREADS=1
cd $R
export GS_PARITY_REPORT=$O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -rf > $O/pytest.txt 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 $O/smoke.txt; exit $rc
