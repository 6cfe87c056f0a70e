#!/bin/bash
# Parity tests + A/B of bench variants (BENCH_VARIANTS="--bcast 0|--bcast 1").
set -u
OUT=gpurun_out
mkdir -p $OUT
export OPENBLAS_NUM_THREADS=1
python -c "import __graft_entry__ as g; g.build()" > $OUT/build.log 2>&1 || { echo "build failed"; exit 2; }
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 900 python -m pytest tests -m gpu -x -q > $OUT/pytest_gpu.log 2>&1; rc=$?
  echo "pytest rc=$rc"; tail -15 $OUT/pytest_gpu.log
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
fi
IFS='|' read -ra VS <<< "${BENCH_VARIANTS:-}"
i=0
for v in "${VS[@]}"; do
  timeout -k 10 300 python bench.py --no-cpu-baseline $v > $OUT/ab_$i.log 2>&1; rc=$?
  echo "variant [$v] rc=$rc"; tail -1 $OUT/ab_$i.log | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(' value %.4g ms/step %.4g frac %.4f kern_ms %.3f' % (d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['kernel_avg_ms']))" 2>/dev/null || tail -3 $OUT/ab_$i.log
  [ $rc -eq 0 ] || exit $rc
  i=$((i+1))
done
