#!/bin/bash
# Round 6: k_sweep_pair with both chains' rho steps in one pass (GS_PAIR_RHO_MERGE) -- bit identity,
# A/B against the per-chain rho steps (libpulsar_gibbs_nomerge.so), the cost model's default vs the
# pair kernel at other chain counts, and one SQ counter pass over the sched-3 headline.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r06l}
mkdir -p $O
export OPENBLAS_NUM_THREADS=1
cd $R
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py \
  -k "two_chains or handoff" > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
ARGS="--no-cpu-baseline --ess 0 --indep 0 --pta none --ecorr 0 --config5 0 --host-stream 0 --warmup 5"
show() { python3 -c "import json; d=json.load(open('$1')); print('$2', 'value %.4e' % d['value'], 'ms %.4f' % d['ms_per_step'], 'kern %.4f' % d['roofline']['kernel_avg_ms'], 'frac %.4f' % d['roofline']['frac'])"; }
for V in merge nomerge merge nomerge; do
  if [ $V = merge ]; then unset GS_LIB_PATH; else export GS_LIB_PATH=$R/pulsar_timing_gibbsspec_amd/libpulsar_gibbs_nomerge.so; fi
  timeout -k 10 170 python3 bench.py $ARGS --steps 40 --sched 3 > $O/ab_$V.json 2> $O/ab_$V.log
  rc=$?; [ $rc -eq 0 ] || { echo "$V rc=$rc"; exit $rc; }
  show $O/ab_$V.json "sched3 $V"
done
unset GS_LIB_PATH
for C in 1024 2048 8192; do
  for SC in 0 3; do
    timeout -k 10 170 python3 bench.py $ARGS --steps 20 --chains $C --sched $SC > $O/c${C}_s$SC.json 2> $O/c${C}_s$SC.log
    rc=$?; [ $rc -eq 0 ] || { echo "c$C s$SC rc=$rc"; exit $rc; }
    show $O/c${C}_s$SC.json "chains $C sched $SC"
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM \
  SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d $O/sq -o run -- python3 $R/bench.py $ARGS --steps 20 --warmup 3 --sched 3 \
  > $O/sq.log 2>&1
rc=$?; echo "sq rc=$rc"; tail -2 $O/sq.log
