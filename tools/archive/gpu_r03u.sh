#!/bin/bash
# r03u: k_bdraw_tiled chain groups per workgroup with the issue priorities on (2 / 3 / 4 / 5)
set -u
export OPENBLAS_NUM_THREADS=1
LIBS="default l2 l3 l5 default l2 l3 l5" PTA=curn_red,curn bash tools/gpu_ab_pta.sh
