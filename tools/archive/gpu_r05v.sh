#!/bin/bash
# r05v: ECORR likelihood kernel time against the chain count (launch-shape cost: 3072 chains = one
# round of 3 waves/SIMD for the shared-operand kernel, 4096 = 1.33 rounds, 6144 = 2)
set -u
out=gpurun_out/r05v; mkdir -p $out
export OPENBLAS_NUM_THREADS=1
for C in 1024 2048 3072 4096 5120 6144 8192; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --pta none --config5 0 --indep 0 --steps 3 --warmup 2 --ecorr-steps 20 --ecorr-chains $C > $out/c$C.json 2> $out/c$C.err || { echo "FAIL $C"; tail -3 $out/c$C.err; exit 3; }
  python -c "
import json;d=json.load(open('$out/c$C.json'));s=d['secondary']
print($C, ' '.join('%s kernel %.4f ms (%.2f us/chain)' % (k, v['roofline']['kernel_avg_ms'], v['roofline']['kernel_avg_ms']*1e3/$C*1e3) for k,v in s.items()))"
done
