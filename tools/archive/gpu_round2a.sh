#!/bin/bash
# Round-2 check: grid-evaluation ceiling probe, the GPU tests, smoke, one default bench run.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd $R
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 tools/probe/grid_probe.hip -o /tmp/grid_probe || exit 2
timeout -k 10 120 /tmp/grid_probe > $O/grid_probe.json || exit 3
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1
echo "pytest rc=$?" >> $O/pytest_gpu.log
tail -3 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; cat $O/smoke.log; exit 4; }
cat $O/smoke.log | tail -1
cp $O/grid_probe.json profiles/grid_probe.json
timeout -k 10 900 python -u bench.py > $O/bench.json 2> $O/bench.err
echo "bench rc=$?"
tail -c 3000 $O/bench.json
