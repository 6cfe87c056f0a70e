#!/bin/bash
# r03z profiles: rocprofv3 kernel trace + stats of the bench command, then the headline's
# FETCH_SIZE / WRITE_SIZE passes (separate runs).
set -u
bash tools/gpu_prof_trace.sh r03z || exit $?
TAG=r03z bash tools/gpu_profile.sh || exit $?
