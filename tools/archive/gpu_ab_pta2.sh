#!/bin/bash
# PTA (configs[3]) A/B of library variants: LIBS="cur name ..." REPS=n
set -u
O=gpurun_out
mkdir -p $O
export OPENBLAS_NUM_THREADS=1
for rep in $(seq ${REPS:-2}); do
  for v in ${LIBS}; do
    if [ "$v" = cur ]; then unset GS_LIB_PATH; else export GS_LIB_PATH=$PWD/pulsar_timing_gibbsspec_amd/libpulsar_gibbs_$v.so; fi
    timeout -k 10 300 python bench.py --no-cpu-baseline --indep 0 --ecorr 0 --config5 0 --host-stream 0 --steps ${STEPS:-100} ${BENCH_ARGS:-} > $O/abp_$v.log 2>&1 || { echo "FAIL $v"; tail -5 $O/abp_$v.log; exit 3; }
    python -c "
import json
d=json.loads(open('$O/abp_$v.log').read().strip().splitlines()[-1])
print('$v', 'head %.4e %.3f' % (d['value'], d['roofline']['kernel_avg_ms']), ' '.join('%s %.4e %.3fms %s' % (k, v['value'], v['ms_per_step'], {kk: round(vv['kernel_avg_ms'], 3) for kk, vv in v.get('kernels', {}).items()}) for k, v in d['secondary'].items()))"
  done
done
