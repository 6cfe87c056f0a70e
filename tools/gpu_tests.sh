#!/bin/bash
# GPU test run: bash tools/gpu_tests.sh <outdir> [pytest selection...]
out=gpurun_out/$1
shift
mkdir -p $out
export GS_PARITY_REPORT=$out
sel="${@:-tests}"
timeout -k 10 500 python -u -m pytest $sel -m gpu -q --timeout 120 --timeout-method thread -rf > $out/pytest.txt 2>&1
rc=$?
tail -5 $out/pytest.txt
exit $rc
