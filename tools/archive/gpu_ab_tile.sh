set -u
mkdir -p gpurun_out
export OPENBLAS_NUM_THREADS=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_tile.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_tile.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for bc in 2 3; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --pta none --bcast $bc > gpurun_out/bench_bc$bc.log 2>&1 || exit 3
  python -c "import json;d=json.loads(open('gpurun_out/bench_bc$bc.log').read().strip().splitlines()[-1]);print($bc, d['value'], d['roofline']['kernel_avg_ms'], d['roofline']['frac'])"
done
