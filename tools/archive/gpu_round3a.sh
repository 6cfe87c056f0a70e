#!/bin/bash
# Round 3: full GPU suite + configs[4] accuracy diagnostic after the double-double prefix.
out=gpurun_out/r03a
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $out/pytest.txt 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 180 python -u tools/accuracy_c5.py > $out/acc_c5.txt 2>&1
echo "acc rc=$?"
