#!/bin/bash
# Round 6: WRITE_SIZE over the same bench command as r06d's FETCH_SIZE pass (ECORR lines: full likelihood
# launches and the incremental Metropolis step kernel, shared and per-chain operands).
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r06e}
mkdir -p $O
export OPENBLAS_NUM_THREADS=1
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/wr -o run -- \
  python3 $R/bench.py --no-cpu-baseline --pta none --config5 0 --indep 0 --steps 2 --warmup 1 \
  --ecorr-steps 2 --ess 0 > $O/wr.json 2> $O/wr.log
echo "wr rc=$?"; tail -3 $O/wr.log
