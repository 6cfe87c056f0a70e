#!/bin/bash
# Grid/PTA tests + the PTA bench lines with per-kernel HIP-event times.
set -u
O=gpurun_out
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_grid_pta.py -q --timeout 200 --timeout-method thread > $O/pytest_grid.log 2>&1
tail -2 $O/pytest_grid.log
timeout -k 10 300 python bench.py --no-cpu-baseline --indep 0 --pta ${PTA:-curn_red,curn} --ecorr 0 --config5 0 \
  --host-stream 0 --steps 20 --warmup 2 --pta-steps ${PTA_STEPS:-50} > $O/bench_pta.json 2> $O/bench_pta.err || { tail -5 $O/bench_pta.err; exit 3; }
python - <<'PY'
import json
d = json.loads(open("gpurun_out/bench_pta.json").read().strip().splitlines()[-1])
for k, v in d["secondary"].items():
    print(k, "%.4e" % v["value"], "%.3f ms/sweep" % v["ms_per_step"],
          {kk: (round(vv["kernel_avg_ms"], 3), round(vv["frac"] or 0, 3)) for kk, vv in v["kernels"].items()})
PY
