#!/bin/bash
# Round 6 profiling call (one gpurun): (1) SQ instruction counters of the shipped headline kernel
# (bench.py's simd_issue reads profiles/sq_headline.json), (2) the ECORR sweep under --kernel-trace
# and then under --pmc with /proc/self/maps written first (tools/ecorr_pmc_probe.py), LAST because
# it is the step that has crashed the host process (nothing runs on the GPU after it).
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r06b}
mkdir -p $O
export OPENBLAS_NUM_THREADS=1
cd /tmp && export TMPDIR=/tmp
ARGS="--no-cpu-baseline --indep 0 --pta none --ecorr 0 --config5 0 --host-stream 0 --ess 0 --steps 20 --warmup 3"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM \
  SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d $O/sq -o run -- python3 $R/bench.py $ARGS > $O/sq.log 2>&1
rc=$?; echo "sq rc=$rc"; tail -2 $O/sq.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python3 $R/tools/ecorr_pmc_probe.py $O/plain 256 > $O/plain.log 2>&1
rc=$?; echo "plain rc=$rc"; tail -2 $O/plain.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- \
  python3 $R/tools/ecorr_pmc_probe.py $O/kt_maps 256 > $O/kt.log 2>&1
rc=$?; echo "kt rc=$rc"; tail -2 $O/kt.log
[ $rc -eq 0 ] || exit $rc
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc -o run -- \
  python3 $R/tools/ecorr_pmc_probe.py $O/pmc_maps 256 > $O/pmc.log 2>&1
echo "pmc rc=$?"; tail -30 $O/pmc.log
