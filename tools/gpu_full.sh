#!/bin/bash
# Full round check: GPU tests, smoke, driver-style bench.  bash tools/gpu_full.sh <outdir> [bench args]
out=gpurun_out/$1
shift
mkdir -p $out
export GS_PARITY_REPORT=$out
timeout -k 10 500 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -rf > $out/pytest.txt 2>&1
rc=$?; tail -3 $out/pytest.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || exit $?
tail -1 $out/smoke.log
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 "$@" > $out/bench.json 2> $out/bench.err || exit $?
python -c "
import json,sys; d=json.load(open('$out/bench.json'))
print('headline', '%.4g'%d['value'], 'frac', '%.3f'%d['roofline']['frac'], 'kernel_ms', '%.3f'%d['roofline']['kernel_avg_ms'], 'ess/s', '%.3g'%d['ess_per_s'])
for k,v in d['secondary'].items(): print(k, '%.4g'%v['value'], v.get('unit'), 'ms/step %.3f'%v['ms_per_step'])
"
