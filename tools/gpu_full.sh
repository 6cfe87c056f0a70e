#!/bin/bash
# The one GPU-session driver (run through gpurun; the library is built beforehand on the CPU
# container and travels in-tree).  bash tools/gpu_full.sh <outdir> [bench args]
#
# Steps, each under its own time limit; a crash / abort / timeout ends the script (no retries):
#   TESTS=1     pytest -m gpu (SEL= a test selection, default tests/)
#   SMOKE=1     __graft_entry__.smoke()
#   BENCH=1     the driver's bench command: bench.py --gpus 1 --steps 20 --warmup 5 [bench args]
#   PROF=0      rocprofv3 --kernel-trace --stats of the same bench command + per-launch durations
#               of the dominant kernels (tools/gpu_prof_trace.sh)
#   PMC=""      kernel-name substrings: FETCH_SIZE / WRITE_SIZE / SQ passes over PMC_ARGS bench
#               arguments, per-dispatch means (tools/gpu_pmc_traffic.sh)
#   AB=""       library variants (csrc/Makefile variant-one) for an interleaved headline A/B
#               (tools/gpu_ab_lib.sh; AB_ARGS extra bench arguments)
# The per-round one-off wrappers of rounds 2-4 are kept in tools/archive/ (the commands behind
# profiles/<round>/SUMMARY.md).
set -u
name=$1
out=gpurun_out/$name
shift
mkdir -p $out
export GS_PARITY_REPORT=$out OPENBLAS_NUM_THREADS=1
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 600 python -u -m pytest ${SEL:-tests} -m gpu -q --timeout 120 --timeout-method thread -rf \
    > $out/pytest.txt 2>&1
  rc=$?; tail -3 $out/pytest.txt
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
fi
if [ "${SMOKE:-1}" = 1 ]; then
  timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || exit $?
  tail -1 $out/smoke.log
fi
if [ "${BENCH:-1}" = 1 ]; then
  timeout -k 10 900 python -u bench.py --gpus 1 --steps 20 --warmup 5 "$@" > $out/bench.json 2> $out/bench.err || exit $?
  python -c "
import json,sys; d=json.load(open('$out/bench.json'))
print('headline', '%.4g'%d['value'], 'frac', '%.3f'%d['roofline']['frac'], 'kernel_ms', '%.3f'%d['roofline']['kernel_avg_ms'], 'ess/s', '%.3g'%d['ess_per_s'])
for k,v in d['secondary'].items(): print(k, '%.4g'%v['value'], v.get('unit'), 'ms/step %.3f'%v['ms_per_step'])
"
fi
if [ "${PROF:-0}" = 1 ]; then
  bash tools/gpu_prof_trace.sh $name "$@" || exit $?
fi
if [ -n "${PMC:-}" ]; then
  TAG=$name KERNELS="$PMC" BENCH_ARGS="${PMC_ARGS:-}" bash tools/gpu_pmc_traffic.sh || exit $?
fi
if [ -n "${AB:-}" ]; then
  LIBS="$AB" BENCH_ARGS="${AB_ARGS:-}" bash tools/gpu_ab_lib.sh 2>&1 | tee $out/ab.txt
fi
