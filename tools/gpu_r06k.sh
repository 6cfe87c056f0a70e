#!/bin/bash
# Round 6: two chains per wavefront (k_sweep_pair, GS_OPT_SWEEP_SCHED = 3) -- bit identity against
# the one-chain kernel, then the headline A/B (cost-model default vs sched 3 vs sched 2) and a
# kernel-trace of the sched-3 headline.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r06k}
mkdir -p $O
export OPENBLAS_NUM_THREADS=1
cd $R
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py \
  -k "two_chains or handoff" > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
ARGS="--no-cpu-baseline --ess 0 --indep 0 --pta none --ecorr 0 --config5 0 --host-stream 0 --steps 20 --warmup 5"
for SC in 0 3 2 3 0; do
  timeout -k 10 170 python3 bench.py $ARGS --sched $SC > $O/bench_s$SC.json 2> $O/bench_s$SC.log
  rc=$?; echo "sched $SC rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python3 -c "import json,sys; d=json.load(open('$O/bench_s$SC.json')); print('sched $SC', d['value'], d['ms_per_step'], d['roofline']['frac'])"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 170 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/bench.py $ARGS --sched 3 \
  > $O/prof_bench.json 2> $O/prof.log
rc=$?; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
find $O/prof -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats.csv \;
find $O/prof -name "*kernel_trace.csv" -exec rm {} \;
head -5 $O/kernel_stats.csv
