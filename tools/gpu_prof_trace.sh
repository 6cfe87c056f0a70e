#!/bin/bash
# rocprofv3 kernel trace + stats of the driver's bench command (no CPU baseline), and the
# per-launch durations of the dominant kernels.  bash tools/gpu_prof_trace.sh <outdir> [bench args]
set -u
out=$GRAFT_REPO_ROOT/gpurun_out/$1
shift
mkdir -p $out
export OPENBLAS_NUM_THREADS=1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $out/prof -o run --output-format csv \
   -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --steps 20 --warmup 5 "$@" > $out/bench_prof.json 2> $out/prof.err; rc=$?
echo "rocprof rc=$rc"
[ $rc -eq 0 ] || { tail -5 $out/prof.err; exit $rc; }
cd $GRAFT_REPO_ROOT
tr=$(find $out/prof -name '*kernel_trace.csv' | head -1)
st=$(find $out/prof -name '*kernel_stats.csv' | head -1)
cp $st $out/kernel_stats.csv
for k in "k_sweep_freespec<" k_sweep_freespec_rm k_bdraw_tiled "k_bdraw<" k_rho_red_cert16 "k_rho_red_cert(" k_rho_red_wave k_hyper_mh k_lnlike_marg k_rho_curn_fast k_rho_curn_sum_wave k_white_syrk k_ecorr_prefix; do
  python tools/launch_stats.py $tr $k
done > $out/launch_stats.log
grep mean $out/launch_stats.log
