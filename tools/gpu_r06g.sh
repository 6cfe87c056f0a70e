#!/bin/bash
# Round 6 closing-style check: the driver's bench command, then the same command under
# rocprofv3 --kernel-trace --stats (the per-kernel averages behind roofline.kernel_avg_ms).
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r06g}
mkdir -p $O
export OPENBLAS_NUM_THREADS=1
cd $R
timeout -k 10 540 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench rc=$rc"; tail -2 $O/bench.err; cp gpurun_out/bench_detail.json $O/bench_detail.json
[ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 540 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
  python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 > $O/prof_bench.json 2> $O/prof_bench.err
echo "prof rc=$?"; tail -2 $O/prof_bench.err
