#!/bin/bash
# r03g: full GPU suite on the 3-wave tiled default, then the CURN line A/B of k_bdraw variants
# (chain-group loop 2 / 4, issue priorities) and the headline.
set -u
mkdir -p gpurun_out/r03g
export OPENBLAS_NUM_THREADS=1
bash tools/gpu_tests.sh r03g || exit $?
LIBS="${PLIBS:-default loop2 loop4 bpr3 default}" PTA=curn bash tools/gpu_ab_pta.sh
