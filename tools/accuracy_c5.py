"""Where does the full-size configs[4] b draw lose accuracy (GPU diagnostic)?
Compares, against the exact long-double draw: numpy fp64 on numpy's TNT, numpy fp64 on the
device's TNT, the device draw on the device's TNT, and the device draw on the exact TNT."""
import sys, os
import numpy as np
import scipy.linalg as sl
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pulsar_timing_gibbsspec_amd import _lib, synthetic
from pulsar_timing_gibbsspec_amd.engine import DeviceModel
from oracle import gibbs_oracle as O
from tests.parity_data import exact_chol_draw_pre, exact_tnt, normwise_rel

d = synthetic.config5_array(n_psr=1, n_toa=int(sys.argv[1]) if len(sys.argv) > 1 else 10000, n_f=100, seed=21)
T, r = d["T"][0], d["r"][0]
N = d["sigma"][0] ** 2
m = T.shape[1]
rng = np.random.default_rng(5)
logrho = rng.uniform(-8.5, -5.0, 100)
ph = 1.0 / np.repeat(10 ** (2 * logrho), 2)
z = rng.standard_normal(m)
phi = np.full(m, 1e-40); phi[d["fidx"]] = ph
order = O.chol_order(m, d["fidx"])
tl = exact_tnt(T, N, r)
bx = exact_chol_draw_pre(tl, phi, z, order)


def np_draw(TNT, dv):
    S = (TNT + np.diag(phi))[np.ix_(order, order)]
    L = np.linalg.cholesky(S)
    y = sl.solve_triangular(L, dv[order], lower=True) + z[order]
    xx = sl.solve_triangular(L.T, y, lower=False)
    b = np.empty(m); b[order] = xx
    return b


ctx = _lib.Context(0, seed=1)
model = DeviceModel(ctx, [T], [N], [r], [d["fidx"]], [d["phiinv_fixed"]])
TNTd, dd = model.tnt_host(0)
TNTn = T.T @ (T / N[:, None]); dn = T.T @ (r / N)
TNTx = np.asarray(tl[0], np.float64); dx = np.asarray(tl[1], np.float64)
out = {"numpy_draw_numpy_tnt": normwise_rel(np_draw(TNTn, dn), bx),
       "numpy_draw_device_tnt": normwise_rel(np_draw(TNTd, dd), bx),
       "numpy_draw_exact_tnt": normwise_rel(np_draw(TNTx, dx), bx),
       "device_tnt_rel_err": float(np.max(np.abs(TNTd - TNTx)) / np.max(np.abs(TNTx))),
       "numpy_tnt_rel_err": float(np.max(np.abs(TNTn - TNTx)) / np.max(np.abs(TNTx)))}
dev = lambda a: torch.as_tensor(np.ascontiguousarray(a), device=ctx.device)
zz = np.zeros((1, model.ldb)); zz[0, :m] = z
b, info = model.bdraw(dev(ph[None]), 1, z=dev(zz))
bd = b.cpu().numpy()[0, :m]
out["device_draw_device_tnt"] = normwise_rel(bd, bx)
fi = np.asarray(d["fidx"]); mi = np.setdiff1d(np.arange(m), fi); sc = np.max(np.abs(bx))
bn = np_draw(TNTn, dn)
out["device_F_part"] = float(np.max(np.abs(bd[fi] - bx[fi])) / sc)
out["device_M_part"] = float(np.max(np.abs(bd[mi] - bx[mi])) / sc)
out["numpy_F_part"] = float(np.max(np.abs(bn[fi] - bx[fi])) / sc)
out["numpy_M_part"] = float(np.max(np.abs(bn[mi] - bx[mi])) / sc)
out["F_rel_own_scale_device"] = float(np.max(np.abs(bd[fi] - bx[fi])) / np.max(np.abs(bx[fi])))
out["F_rel_own_scale_numpy"] = float(np.max(np.abs(bn[fi] - bx[fi])) / np.max(np.abs(bx[fi])))
# device draw from the exact (fp64-rounded) TNT: overwrite TNT/d, redo the prefix only
lo = lambda a, h: np.asarray(a - np.asarray(h, np.longdouble), np.float64)  # noqa: E731
TNT_dev_hi, TNT_dev_lo = model.TNT.clone(), model.TNT_lo.clone()
out["device_tnt_dd_rel_err"] = float(np.max(np.abs(
    np.asarray(TNT_dev_hi.cpu().numpy(), np.longdouble).reshape(m, m) + TNT_dev_lo.cpu().numpy().reshape(m, m)
    - tl[0])) / np.max(np.abs(np.asarray(tl[0], np.float64))))
model.TNT.copy_(torch.as_tensor(TNTx.ravel(), device=ctx.device))
model.TNT_lo.copy_(torch.as_tensor(lo(tl[0], TNTx).ravel(), device=ctx.device))
model.d.copy_(torch.as_tensor(dx, device=ctx.device))
model.d_lo.copy_(torch.as_tensor(lo(tl[1], dx), device=ctx.device))
model.prefix()
b2, _ = model.bdraw(dev(ph[None]), 1, z=dev(zz))
out["device_draw_exact_tnt"] = normwise_rel(b2.cpu().numpy()[0, :m], bx)
print({k: float("%.3g" % v) for k, v in out.items()})
# mean only (z = 0), the device on the exact TNT (set above); numpy on its own and on the exact TNT
z0 = np.zeros((1, model.ldb))
model.TNT.copy_(TNT_dev_hi)
model.TNT_lo.copy_(TNT_dev_lo)
model.prefix()
b0, _ = model.bdraw(dev(ph[None]), 1, z=dev(z0))
bx0 = exact_chol_draw_pre(tl, phi, np.zeros(m), order)
sc = np.max(np.abs(bx))
b0d = b0.cpu().numpy()[0, :m]
res = {"mean_only_F": float(np.max(np.abs(b0d[fi] - bx0[fi])) / sc),
       "mean_only_M": float(np.max(np.abs(b0d[mi] - bx0[mi])) / sc)}
zsave = z.copy(); z[:] = 0.0
bn0 = np_draw(TNTn, dn); z[:] = zsave
res["numpy_mean_only_F"] = float(np.max(np.abs(bn0[fi] - bx0[fi])) / sc)
res["numpy_mean_only_M"] = float(np.max(np.abs(bn0[mi] - bx0[mi])) / sc)
z[:] = 0.0
bnx = np_draw(TNTx, dx); z[:] = zsave           # numpy on the exact TNT (as the device run above)
res["numpy_exact_tnt_mean_only_F"] = float(np.max(np.abs(bnx[fi] - bx0[fi])) / sc)
res["numpy_exact_tnt_mean_only_M"] = float(np.max(np.abs(bnx[mi] - bx0[mi])) / sc)
print({k: float("%.3g" % v) for k, v in res.items()})
