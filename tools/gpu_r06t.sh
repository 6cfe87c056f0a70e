#!/bin/bash
# Round 6 closing-style check (k_sweep_pair headline): the driver's bench command, then the same command under
# rocprofv3 --kernel-trace --stats (the per-kernel averages behind roofline.kernel_avg_ms).  The kernel
# trace itself (~100 MB) is reduced to launch_stats.txt (tools/launch_stats.py) and deleted, so the
# merged gpurun_out/ stays under the 64 MiB copy-back limit.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r06t}
mkdir -p $O
export OPENBLAS_NUM_THREADS=1
cd $R
timeout -k 10 540 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench rc=$rc"; tail -2 $O/bench.err; cp gpurun_out/bench_detail.json $O/bench_detail.json
[ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 540 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
  python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 > $O/prof_bench.json 2> $O/prof_bench.err
rc=$?; echo "prof rc=$rc"; tail -2 $O/prof_bench.err
cd $R
KT=$(find $O/prof -name "*kernel_trace.csv" | head -1)
python3 tools/launch_stats.py "$KT" "k_sweep_pair<4>" > $O/launch_stats.txt 2>&1
for k in k_bdraw_tiled k_rho_red_cert16 k_rho_curn_fast k_hyper_mh k_white_syrk "k_ecorr_prefix<5, true, false, true>"; do
  python3 tools/launch_stats.py "$KT" "$k" | cut -c1-600 >> $O/launch_stats.txt 2>&1
done
echo "stats rc=$?"; cut -c1-300 $O/launch_stats.txt
find $O/prof -name "*kernel_trace.csv" -delete
rm -rf $R/gpurun_out/ess_rows
du -sh $O
