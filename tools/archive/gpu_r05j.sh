#!/bin/bash
# r05j: rehearse the N = 2 bench path (two ranks on the one GPU over gloo) incl. the pulsar-sharded
# PTA lines (curn, curn_red, curn_plred) -- what the driver's multi-GPU scaling run executes over RCCL
set -u
mkdir -p gpurun_out/r05j
export GS_DIST_BACKEND=gloo OPENBLAS_NUM_THREADS=1
timeout -k 10 900 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 \
  bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu-baseline --indep 0 --ecorr 0 --config5 0 --pta-steps 20 --pta-ess-sweeps 0 \
  --ess-sweeps 200 > gpurun_out/r05j/bench2.json 2> gpurun_out/r05j/bench2.err; rc=$?
echo "rc=$rc"; tail -3 gpurun_out/r05j/bench2.err
python - <<'PY'
import json
d = json.loads(open("gpurun_out/r05j/bench2.json").read().strip().splitlines()[-1])
print("n_gpus", d["n_gpus"], "value %.4g" % d["value"])
for k, v in d["secondary"].items():
    print(k, "%.4g" % v["value"], v.get("sharding"), v.get("scaling"))
PY
