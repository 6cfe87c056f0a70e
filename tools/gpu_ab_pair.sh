#!/bin/bash
# A/B of library variants on the headline (default cost model -> k_sweep_pair), interleaved:
# LIBS="default diag0 ..." REPS=2 bash tools/gpu_ab_pair.sh
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-ab_pair}
mkdir -p $O
export OPENBLAS_NUM_THREADS=1
cd $R
ARGS="--no-cpu-baseline --ess 0 --indep 0 --pta none --ecorr 0 --config5 0 --host-stream 0 --warmup 5 --steps ${STEPS:-40} ${BENCH_ARGS:-}"
for r in $(seq ${REPS:-2}); do
  for v in ${LIBS:-default}; do
    if [ "$v" = default ]; then unset GS_LIB_PATH; else export GS_LIB_PATH=$R/pulsar_timing_gibbsspec_amd/libpulsar_gibbs_$v.so; fi
    timeout -k 10 170 python3 bench.py $ARGS > $O/${v}_$r.json 2> $O/${v}_$r.log
    rc=$?; [ $rc -eq 0 ] || { echo "$v rc=$rc"; tail -3 $O/${v}_$r.log; exit $rc; }
    python3 -c "import json; d=json.load(open('$O/${v}_$r.json')); print('$v', 'value %.4e' % d['value'], 'ms %.4f' % d['ms_per_step'], 'kern %.4f' % d['roofline']['kernel_avg_ms'], d['roofline']['kernel'])"
  done
done
