#!/bin/bash
# Round 6: (1) the ECORR probe at the bench's 4096 chains without a profiler; (2) a 2-rank rehearsal of
# bench.py on the one GPU (GS_DIST_BACKEND=gloo, ranks sharing the device: the N > 1 code paths incl.
# the pulsar-sharded curn_plred line); (3) LAST, the ECORR probe at 4096 chains under rocprofv3 --pmc
# (the configuration that crashed in round 5), /proc/self/maps written before the first ECORR launch.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r06c}
mkdir -p $O
export OPENBLAS_NUM_THREADS=1
timeout -k 10 120 python3 $R/tools/ecorr_pmc_probe.py $O/plain 4096 > $O/plain.log 2>&1
rc=$?; echo "plain rc=$rc"; tail -2 $O/plain.log
[ $rc -eq 0 ] || exit $rc
GS_DIST_BACKEND=gloo timeout -k 10 420 python3 $R/bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline --ess 0 \
  --indep-steps 100 --pta curn_plred --pta-steps 20 --ecorr-steps 2 --c5-steps 1 > $O/n2.json 2> $O/n2.err
rc=$?; echo "n2 rc=$rc"; tail -3 $O/n2.err; wc -c $O/n2.json
[ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc -o run -- \
  python3 $R/tools/ecorr_pmc_probe.py $O/pmc_maps 4096 > $O/pmc.log 2>&1
echo "pmc rc=$?"; tail -40 $O/pmc.log
