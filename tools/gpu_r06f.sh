#!/bin/bash
# Round 6: the GPU suite (incl. the 45-pulsar curn_plred KS and mixing tests against the new reference
# runs), then an A/B of k_bdraw_tiled variants on the PTA lines: default (next item's phiinv / gate flag
# prefetched), nopf (GS_BDRAW_PREFETCH=0), noload (cost probe: no phiinv / gate loads, wrong draws).
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r06f}
mkdir -p $O
export OPENBLAS_NUM_THREADS=1
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -4 $O/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u -m pytest tests/test_gpu_ks_pta.py -m gpu -v --timeout 300 --timeout-method thread > $O/ks.log 2>&1
echo "ks rc=$?"; grep -E "PASS|FAIL|SKIP" $O/ks.log | head
for v in default nopf noload default nopf; do
  if [ "$v" = default ]; then unset GS_LIB_PATH; else export GS_LIB_PATH=$R/pulsar_timing_gibbsspec_amd/libpulsar_gibbs_$v.so; fi
  timeout -k 10 300 python bench.py --no-cpu-baseline --ess 0 --indep 0 --ecorr 0 --config5 0 --host-stream 0 \
    --steps 20 --warmup 5 --pta curn,curn_plred --pta-steps 300 > $O/ab_$v.json 2> $O/ab_$v.err || { echo "FAIL $v"; tail -5 $O/ab_$v.err; exit 3; }
  python -c "import json;d=json.loads(open('$O/ab_$v.json').read().strip().splitlines()[-1]);s=d['secondary'];print('$v', {k:(v['value'], v['roofline'].get('kernel'), v['roofline'].get('kernel_avg_ms')) for k,v in s.items()})"
done
