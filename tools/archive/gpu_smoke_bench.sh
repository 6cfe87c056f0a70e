#!/bin/bash
# smoke + driver-style bench: bash tools/gpu_smoke_bench.sh <outdir> [bench args]
out=gpurun_out/$1
shift
mkdir -p $out
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || exit $?
tail -1 $out/smoke.log
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 "$@" > $out/bench.json 2> $out/bench.err || exit $?
python tools/bench_summary.py $out/bench.json
