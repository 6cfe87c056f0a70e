#!/bin/bash
# Round 6: gs_bdraw_tiled on two chains per wave (k_bdraw_pair).  Its bit-identity tests, the whole GPU
# suite, then the PTA curn / curn_red lines with the cost model's pair draw against a library whose
# cost model never picks it (libpulsar_gibbs_bp0.so), interleaved.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r06r}
mkdir -p $O
export OPENBLAS_NUM_THREADS=1
cd $R
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_bdraw_pair.py > $O/pytest_pair.log 2>&1
rc=$?; echo "pair tests rc=$rc"; tail -3 $O/pytest_pair.log; [ $rc -eq 0 ] || exit $rc
export GS_PARITY_REPORT=$O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -rf > $O/pytest.txt 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.txt; [ $rc -eq 0 ] || exit $rc
ARGS="--no-cpu-baseline --ess 0 --indep 0 --pta curn,curn_red --ecorr 0 --config5 0 --host-stream 0 --steps 20 --warmup 5"
for r in 1 2; do
  for v in default bp0; do
    if [ $v = default ]; then unset GS_LIB_PATH; else export GS_LIB_PATH=$R/pulsar_timing_gibbsspec_amd/libpulsar_gibbs_$v.so; fi
    timeout -k 10 300 python3 bench.py $ARGS > $O/${v}_$r.json 2> $O/${v}_$r.log
    rc=$?; [ $rc -eq 0 ] || { echo "$v rc=$rc"; tail -3 $O/${v}_$r.log; exit $rc; }
    GS_DETAIL=$O/bench_detail.json python3 - <<PY
import json
d=json.load(open('$O/${v}_$r.json'))
for k, v in d.get('secondary', {}).items():
    if k.startswith('curn'):
        print('$v', k, 'value %.4e' % v['value'], 'ms %.4f' % v['ms_per_step'], v.get('roofline'))
PY
  done
done
