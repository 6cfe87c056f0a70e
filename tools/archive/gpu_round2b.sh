#!/bin/bash
# GPU tests + headline-only bench (kernel time of k_sweep_freespec) after a kernel change.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd $R
export GS_PARITY_REPORT=$O/parity
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread ${PYTEST_ARGS:-} > $O/pytest_gpu.log 2>&1
echo "pytest rc=$?" >> $O/pytest_gpu.log
tail -3 $O/pytest_gpu.log
grep -E "FAILED|Error" $O/pytest_gpu.log | head -20
timeout -k 10 300 python -u bench.py --no-cpu-baseline --indep 0 --pta none --ecorr 0 --config5 0 --host-stream 0 > $O/bench_head.json 2> $O/bench_head.err
echo "bench rc=$?"
python -c "
import json; d=json.loads(open('$O/bench_head.json').read().strip().splitlines()[-1])
print('value', d['value'], 'kernel_ms', d['roofline']['kernel_avg_ms'], 'frac', d['roofline']['frac'])"
