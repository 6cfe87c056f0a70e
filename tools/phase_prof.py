"""Per-phase cycle breakdown of the tile b-draw inside the fused sweep kernel.

Needs the GS_PHASE_PROF variant: make -C pulsar_timing_gibbsspec_amd/csrc variant NAME=phase
EXTRA="-DGS_TILE_MINW=2 -DGS_PHASE_PROF"; run with GS_LIB_PATH pointing at it.
"""
import ctypes
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pulsar_timing_gibbsspec_amd import _lib, synthetic  # noqa: E402
from pulsar_timing_gibbsspec_amd.engine import DeviceModel, FreeSpectrumChains  # noqa: E402

C = int(os.environ.get("CHAINS", "4096"))
S = 100
pta = synthetic.single_pulsar_pta("J1713+0747", seed=0)
T, N, r = pta.get_basis()[0], pta.get_ndiag({})[0], pta.get_residuals()[0]
ctx = _lib.Context(0, seed=1)
model = DeviceModel(ctx, [T], [N], [r], [np.arange(60)], [np.full(T.shape[1] - 60, 1e-40)])
run = FreeSpectrumChains(model, 1e-18, 1e-8, C, np.random.default_rng(0).uniform(-9, -4, (C, 30)))
fn = ctx.lib.gs_debug_phase_cycles
fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
buf = (ctypes.c_ulonglong * 8)()
run.run(S, record=False)
torch.cuda.synchronize()
fn(buf, 1)
t0 = time.perf_counter()
run.run(S, record=False)
torch.cuda.synchronize()
el = time.perf_counter() - t0
fn(buf, 0)
names = ["load+phi", "diag factor", "trsm+update", "forward", "backward", "fixed block", "record+rho+gate", "rng+phinv"]
tot = sum(buf[i] for i in range(8))
draws = C * S
print(f"chains {C} sweeps {S} launch {el*1e3:.2f} ms; per wave per draw cycles:")
for i, n in enumerate(names):
    print(f"  {n:24s} {buf[i] / draws:10.0f}  {100 * buf[i] / tot:5.1f} %")
print(f"  {'sum':24s} {tot / draws:10.0f}")
