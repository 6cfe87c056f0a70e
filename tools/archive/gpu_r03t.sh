#!/bin/bash
# r03t: SQ issue / stall counters of the headline's hand-off sweep (one --pmc pass of 8 SQ counters)
set -u
TAG=_r03t bash tools/gpu_pmc_sq.sh || exit $?
