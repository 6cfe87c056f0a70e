#!/bin/bash
# r03s: PMC traffic of the headline's hand-off sweep (12-wave workgroups: 256 x 768 work-items)
set -u
TAG=r03s GRID=196608 bash tools/gpu_profile.sh || exit $?
