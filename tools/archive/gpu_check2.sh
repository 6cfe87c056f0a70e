#!/bin/bash
# Full GPU tests + the PTA bench lines (per-kernel times).
set -u
O=gpurun_out
mkdir -p $O
export GS_PARITY_REPORT=$O/parity
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1
echo "pytest rc=$?"; tail -2 $O/pytest_gpu.log; grep -E "^E  |FAILED" $O/pytest_gpu.log | head -10
bash tools/gpu_pta_check.sh | tail -3
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 tools/probe/grid_probe.hip -o /tmp/grid_probe && timeout -k 10 60 /tmp/grid_probe > $O/grid_probe.json && cat $O/grid_probe.json
