#!/bin/bash
# Headline A/B of library variants libpulsar_gibbs_<name>.so ("cur" = the in-tree build),
# REPS interleaved repetitions on one box.
set -u
O=gpurun_out
mkdir -p $O
export OPENBLAS_NUM_THREADS=1
for rep in $(seq ${REPS:-2}); do
  for v in ${LIBS}; do
    if [ "$v" = cur ]; then unset GS_LIB_PATH; else export GS_LIB_PATH=$PWD/pulsar_timing_gibbsspec_amd/libpulsar_gibbs_$v.so; fi
    timeout -k 10 300 python bench.py --no-cpu-baseline --pta none --config5 0 --ecorr 0 --indep ${INDEP:-0} --steps ${STEPS:-200} --warmup 10 ${BENCH_ARGS:-} > $O/abv_$v.log 2>&1 || { echo "FAIL $v"; tail -5 $O/abv_$v.log; exit 3; }
    python -c "import json;d=json.loads(open('$O/abv_$v.log').read().strip().splitlines()[-1]);s=d.get('secondary',{});print('$v', 'value %.4e' % d['value'], 'kernel ms/launch %.3f' % d['roofline']['kernel_avg_ms'], 'frac %.4f' % d['roofline']['frac'], {k:'%.4e'%v['value'] for k,v in s.items()})"
  done
done
