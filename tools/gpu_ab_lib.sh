#!/bin/bash
# A/B of library variants (csrc/Makefile `variant` target) on the headline bench.
# LIBS="default minw2 ..." CHAINS="4096 ..." bash tools/gpu_ab_lib.sh
set -u
mkdir -p gpurun_out
export OPENBLAS_NUM_THREADS=1
for v in ${LIBS:-default}; do
  if [ "$v" = default ]; then unset GS_LIB_PATH; else export GS_LIB_PATH=$PWD/pulsar_timing_gibbsspec_amd/libpulsar_gibbs_$v.so; fi
  for C in ${CHAINS:-4096}; do
    timeout -k 10 300 python bench.py --no-cpu-baseline --pta ${PTA:-none} --config5 ${C5:-0} --chains $C --steps ${STEPS:-300} --warmup 20 ${BENCH_ARGS:-} > gpurun_out/ab_${v}_c$C.log 2>&1 || { echo "FAIL $v $C"; tail -5 gpurun_out/ab_${v}_c$C.log; exit 3; }
    python -c "import json;d=json.loads(open('gpurun_out/ab_${v}_c$C.log').read().strip().splitlines()[-1]);s=d.get('secondary',{});print('$v', 'chains', $C, 'value %.4e' % d['value'], 'kernel ms/launch %.3f' % d['roofline']['kernel_avg_ms'], 'frac %.4f' % d['roofline']['frac'], {k:'%.4e'%v['value'] for k,v in s.items()})"
  done
done
