set -u
mkdir -p gpurun_out
for bc in ${BCS:-3}; do
for C in ${CHAINS:-1024 2048 3072 4096 6144}; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --pta none --bcast $bc --chains $C --steps 200 --warmup 20 > gpurun_out/bench_c$C.log 2>&1 || exit 3
  python -c "import json;d=json.loads(open('gpurun_out/bench_c$C.log').read().strip().splitlines()[-1]);print('bc', $bc, 'chains', $C, 'value %.3e' % d['value'], 'kernel ms/100sw %.3f' % d['roofline']['kernel_avg_ms'], 'frac %.3f' % d['roofline']['frac'])"
done
done
