#!/bin/bash
# r03l: k_bdraw_tiled knobs on the PTA lines: issue priorities (bpr), 3 / 6 chain groups per workgroup
set -u
export OPENBLAS_NUM_THREADS=1
LIBS="default bpr l3 l6 default bpr l3 l6" PTA=curn_red,curn bash tools/gpu_ab_pta.sh
