set -u
export OPENBLAS_NUM_THREADS=1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_c5 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --pta none --steps 100 --warmup 10 > $GRAFT_REPO_ROOT/gpurun_out/prof_c5.log 2>&1; rc=$?
echo rc=$rc
cut -c1-160 $GRAFT_REPO_ROOT/gpurun_out/prof_c5/run_kernel_stats.csv | head -14
exit $rc
