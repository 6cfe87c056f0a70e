#!/bin/bash
# A/B of library variants on the PTA lines (per-kernel HIP-event times) and the headline.
# LIBS="default scr400" bash tools/gpu_ab_pta.sh
set -u
mkdir -p gpurun_out
export OPENBLAS_NUM_THREADS=1
for v in ${LIBS:-default}; do
  if [ "$v" = default ]; then unset GS_LIB_PATH; else export GS_LIB_PATH=$PWD/pulsar_timing_gibbsspec_amd/libpulsar_gibbs_$v.so; fi
  timeout -k 10 300 python bench.py --no-cpu-baseline --indep 0 --pta ${PTA:-curn_red,curn} --ecorr 0 --config5 0 \
    --host-stream 0 --steps ${STEPS:-100} --warmup 10 --pta-steps ${PTA_STEPS:-50} > gpurun_out/abp_$v.json 2> gpurun_out/abp_$v.err || { echo "FAIL $v"; tail -5 gpurun_out/abp_$v.err; exit 3; }
  python - "$v" <<'PY'
import json, sys
d = json.loads(open("gpurun_out/abp_%s.json" % sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[1], "headline %.4e %.3f ms/launch" % (d["value"], d["roofline"]["kernel_avg_ms"]))
for k, v in d["secondary"].items():
    print("  ", k, "%.4e" % v["value"], {kk: round(vv["kernel_avg_ms"], 3) for kk, vv in v["kernels"].items()})
PY
done
