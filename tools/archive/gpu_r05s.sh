#!/bin/bash
# r05s: r05q's FETCH_SIZE pass over the ECORR lines died in the host (SIGSEGV in the launch after the
# first k_ecorr_prefix dispatch).  The same pass with the pre-change ECORR kernels (ecold) first, then
# with the current library (last: a crash ends the call).  Kernel trace on, headline-only otherwise.
set -u
R=$GRAFT_REPO_ROOT
out=$R/gpurun_out/r05s; mkdir -p $out
export OPENBLAS_NUM_THREADS=1
ARGS="--no-cpu-baseline --pta none --config5 0 --indep 0 --steps 2 --warmup 1 --ecorr-steps 2"
cd /tmp && export TMPDIR=/tmp
GS_LIB_PATH=$R/pulsar_timing_gibbsspec_amd/libpulsar_gibbs_ecold.so timeout -s KILL 170 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $out/old -o run -- python3 $R/bench.py $ARGS > $out/old.log 2>&1; rc=$?
echo "ecold fetch rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 170 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $out/new -o run -- python3 $R/bench.py $ARGS > $out/new.log 2>&1; rc=$?
echo "new fetch rc=$rc"; exit $rc
