#!/bin/bash
# Round 6: SQ instruction counters of the shipped headline kernel (k_sweep_pair, after the interleaved
# solves and the live-row elimination) -> tools/sq_summary.py -> profiles/sq_headline.json
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r06u}
mkdir -p $O
export OPENBLAS_NUM_THREADS=1
cd /tmp && export TMPDIR=/tmp
ARGS="--no-cpu-baseline --indep 0 --pta none --ecorr 0 --config5 0 --host-stream 0 --ess 0 --steps 20 --warmup 3"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM \
  SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d $O/sq -o run -- python3 $R/bench.py $ARGS > $O/sq.log 2>&1
rc=$?; echo "sq rc=$rc"; tail -1 $O/sq.log
