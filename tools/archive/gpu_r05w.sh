#!/bin/bash
# r05w: SQ counters of the ECORR likelihood kernel through a standalone driver (tools/ecorr_probe.py;
# the bench's ECORR lines crash rocprofv3's PMC mode, r05s), and of the headline kernel for scale.
set -u
R=$GRAFT_REPO_ROOT
export OPENBLAS_NUM_THREADS=1
mkdir -p $R/gpurun_out/r05w
timeout -k 10 300 python -u -m pytest tests/test_gpu_ecorr.py tests/test_gpu_white.py -q --timeout 120 --timeout-method thread -rf > $R/gpurun_out/r05w/pytest.txt 2>&1
rc=$?; tail -3 $R/gpurun_out/r05w/pytest.txt; [ $rc -eq 0 ] || exit $rc
# A/B: the epilogue's logs by gs_log_pos (default) against libm's (ecprev)
for v in default ecprev default ecprev; do
  if [ "$v" = default ]; then unset GS_LIB_PATH; else export GS_LIB_PATH=$PWD/pulsar_timing_gibbsspec_amd/libpulsar_gibbs_$v.so; fi
  timeout -k 10 300 python bench.py --no-cpu-baseline --pta none --config5 0 --indep 0 --steps 3 --warmup 2 --ecorr-steps 40 > $R/gpurun_out/r05w/ab_$v.log 2>/dev/null || { echo "FAIL $v"; exit 3; }
  python -c "
import json;d=json.loads(open('$R/gpurun_out/r05w/ab_$v.log').read().strip().splitlines()[-1]);s=d['secondary']
print('$v', ' '.join('%s %.4e ms/step %.4f kernel %.4f' % (k, v['value'], v['ms_per_step'], v['roofline']['kernel_avg_ms']) for k,v in s.items()))"
done
unset GS_LIB_PATH
timeout -k 10 120 python tools/ecorr_probe.py 4096 20 || exit $?
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU"
TAG=ec KERNELS="k_ecorr_prefix" SQ_COUNTERS="$SQ" bash tools/gpu_pmc_kernel.sh tools/ecorr_probe.py 4096 20 > $R/gpurun_out/r05w/ec.txt 2>&1; rc=$?
cat $R/gpurun_out/r05w/ec.txt; [ $rc -eq 0 ] || exit $rc
TAG=hd KERNELS="k_sweep_freespec<60, 0, 12" SQ_COUNTERS="$SQ" bash tools/gpu_pmc_kernel.sh bench.py --no-cpu-baseline --pta none --config5 0 --indep 0 --ecorr 0 --steps 5 --warmup 2 --ess-sweeps 100 > $R/gpurun_out/r05w/hd.txt 2>&1; rc=$?
cat $R/gpurun_out/r05w/hd.txt; exit $rc
