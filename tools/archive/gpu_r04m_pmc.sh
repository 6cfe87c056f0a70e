#!/bin/bash
# r04m: PMC traffic of the headline's hand-off sweep after the SGPR wave index (12-wave workgroups:
# 256 x 768 work-items), trace + FETCH_SIZE + WRITE_SIZE passes of a short headline-only bench
set -u
TAG=r04m GRID=196608 HEAD_LAUNCHES=6 BENCH_ARGS="--indep 0 --ecorr 0 --host-stream 0 --steps 5 --warmup 1 --ess-sweeps 100 --cpu-ess 0" \
  bash tools/gpu_profile.sh || exit $?
