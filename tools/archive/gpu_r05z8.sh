#!/bin/bash
# r05z8: rehearse the N = 2 bench path (two ranks on the one GPU over gloo) after the round's ECORR
# changes: headline, indep (pulsar-sharded), the PTA lines (chain- and pulsar-sharded), both ECORR lines
set -u
mkdir -p gpurun_out/r05z8
export GS_DIST_BACKEND=gloo OPENBLAS_NUM_THREADS=1
timeout -k 10 900 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29513 \
  bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu-baseline --config5 0 --indep-steps 100 --pta-steps 20 --pta-ess-sweeps 0 \
  --ess-sweeps 200 --ecorr-steps 4 > gpurun_out/r05z8/bench2.json 2> gpurun_out/r05z8/bench2.err; rc=$?
echo "rc=$rc"; tail -3 gpurun_out/r05z8/bench2.err
[ $rc -eq 0 ] || exit $rc
python - <<'PY'
import json
d = json.loads(open("gpurun_out/r05z8/bench2.json").read().strip().splitlines()[-1])
print("n_gpus", d["n_gpus"], "value %.4g" % d["value"])
for k, v in d["secondary"].items():
    print(k, "%.4g" % v["value"], v.get("sharding"), v.get("scaling"), v.get("n_gpus"))
PY
