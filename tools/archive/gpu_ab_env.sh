#!/bin/bash
# A/B of a run-time knob (env VAR, values VALS) on the PTA lines: bash tools/gpu_ab_env.sh VAR "v1 v2 ..." [pta]
set -u
VAR=$1; VALS=$2; PTA=${3:-curn,curn_red}
mkdir -p gpurun_out/abenv
export OPENBLAS_NUM_THREADS=1
for v in $VALS; do
  env $VAR=$v timeout -k 10 300 python bench.py --no-cpu-baseline --steps 3 --warmup 1 --indep 0 --config5 0 --ecorr 0 \
    --pta $PTA --pta-ess-sweeps 0 --ess-sweeps 100 --cpu-ess 0 > gpurun_out/abenv/$VAR-$v.json 2> gpurun_out/abenv/$VAR-$v.err || exit $?
  python -c "
import json; d=json.load(open('gpurun_out/abenv/$VAR-$v.json'))
print('$VAR=$v', {k: ('%.4e' % v['value'], round(v['ms_per_step'], 4), {kk: round(vv['kernel_avg_ms'], 4) for kk, vv in v.get('kernels', {}).items()}) for k, v in d['secondary'].items()})"
done
