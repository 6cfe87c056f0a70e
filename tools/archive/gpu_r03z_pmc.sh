#!/bin/bash
# r03z PMC passes: CURN k_bdraw_tiled, ECORR likelihood kernels (FETCH_SIZE / WRITE_SIZE, separate runs)
set -u
bash tools/gpu_pmc_curn.sh || exit $?
bash tools/gpu_pmc_ecorr.sh || exit $?
