import os, sys
for v in ("OPENBLAS_NUM_THREADS", "OMP_NUM_THREADS", "MKL_NUM_THREADS"):
    os.environ[v] = "1"
sys.path.insert(0, os.getcwd())
import numpy as np, torch
from pulsar_timing_gibbsspec_amd import _lib
from pulsar_timing_gibbsspec_amd.engine import DeviceModel, FreeSpectrumChains
from tests.conftest import golden
from tests.parity_data import normwise_rel, single_replay
g = golden("single_j1713.npz"); R = single_replay(g)
dev = lambda a: torch.as_tensor(np.ascontiguousarray(a), dtype=torch.float64, device="cuda")
for n in (1, 2, 3, 5, 10, 20, 40):
    ctx = _lib.Context(0, seed=7)
    model = DeviceModel(ctx, [g["T"]], [g["Nvec"]], [g["r"]], [R["gwid"]], [np.full(R["n_tm"], 1e-40)])
    run = FreeSpectrumChains(model, R["rhomin"], R["rhomax"], 1, g["x0"])
    xr, br = run.run(n + 1, z0_inj=dev(R["zc"][:1]), z_inj=dev(R["zc"][1:n + 2][:, None]), u_inj=dev(g["U"][:n + 1][:, None]))
    xr, br = xr.cpu().numpy()[:, 0], br.cpu().numpy()[:, 0]
    per = [normwise_rel(br[i:i+1], g["bchain"][i:i+1]) for i in range(1, n + 1)]
    print(n, "chain %.2e" % normwise_rel(xr, g["chain"][:n + 1]), "b %.2e" % normwise_rel(br[1:], g["bchain"][1:n + 1]), "per-draw max %.2e" % max(per), "first %.2e" % per[0])
# every draw vs the exact (long double) Cholesky draw at the device's own state
from oracle import gibbs_oracle as O
from tests.parity_data import exact_chol_draw_pre, exact_tnt
n = 40
ctx = _lib.Context(0, seed=7)
model = DeviceModel(ctx, [g["T"]], [g["Nvec"]], [g["r"]], [R["gwid"]], [np.full(R["n_tm"], 1e-40)])
run = FreeSpectrumChains(model, R["rhomin"], R["rhomax"], 1, g["x0"])
xr, br = run.run(n, z0_inj=dev(R["zc"][:1]), z_inj=dev(R["zc"][1:n + 1][:, None]), u_inj=dev(g["U"][:n][:, None]))
xr, br = xr.cpu().numpy()[:, 0], br.cpu().numpy()[:, 0]
m = g["T"].shape[1]
tl = exact_tnt(g["T"], g["Nvec"], g["r"])
order = O.chol_order(m, R["gwid"])
errs = []
for i in range(1, n):
    ph = O.phiinv_single(xr[i], R["n_tm"])
    errs.append(normwise_rel(br[i], exact_chol_draw_pre(tl, ph, R["zc"][i], order)))
print("per-draw vs exact: max %.2e median %.2e" % (max(errs), float(np.median(errs))))
