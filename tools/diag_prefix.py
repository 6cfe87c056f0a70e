"""Accuracy diagnosis of the device TNT / prefix / b draw for one pulsar of the configs[2]
array against numpy and x87 long double (run on the GPU box: python tools/diag_prefix.py P)."""
import os
import sys

os.environ["OPENBLAS_NUM_THREADS"] = "1"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from oracle import gibbs_oracle as O  # noqa: E402
from pulsar_timing_gibbsspec_amd import _lib, synthetic  # noqa: E402
from pulsar_timing_gibbsspec_amd.engine import DeviceModel  # noqa: E402
from tests.parity_data import exact_chol_draw_pre, exact_tnt, normwise_rel  # noqa: E402


def rel(a, b):
    return float(np.max(np.abs(np.asarray(a, float) - np.asarray(b, float))) / np.max(np.abs(np.asarray(b, float))))


def main(p):
    pt = synthetic.pulsar_ptas(synthetic.array_pta(kind="indep", seed=0))[p]
    T, N, r = pt.get_basis()[0], pt.get_ndiag({})[0], pt.get_residuals()[0]
    m = T.shape[1]
    gw = np.arange(60)
    ctx = _lib.Context(0, seed=1)
    model = DeviceModel(ctx, [T], [N], [r], [gw], [np.full(m - 60, 1e-40)])
    TNTd, dd = model.tnt_host(0)
    TNTn, dn = O.tnt(T, N, r)
    tl, dl = exact_tnt(T, N, r)
    print(f"pulsar {p} {pt.pulsars[0]} T {T.shape}")
    print(f"TNT rel err: device {rel(TNTd, tl):.2e}  numpy {rel(TNTn, tl):.2e};  d: device {rel(dd, dl):.2e} numpy {rel(dn, dl):.2e}")
    # prefix blocks vs the long-double prefix
    L_ = np.longdouble
    Mi, Fi = np.arange(60, m), gw
    A = tl[np.ix_(Mi, Mi)].copy()
    A[np.diag_indices_from(A)] += L_(1e-40)
    n = A.shape[0]
    Lm = np.zeros_like(A)
    for k in range(n):
        v = A[k:, k] - Lm[k:, :k] @ Lm[k, :k]
        Lm[k, k] = np.sqrt(v[0])
        Lm[k + 1:, k] = v[1:] / Lm[k, k]
    W = np.zeros((n, 60), dtype=L_)
    B = tl[np.ix_(Mi, Fi)]
    for i in range(n):
        W[i] = (B[i] - Lm[i, :i] @ W[:i]) / Lm[i, i]
    S0x = tl[np.ix_(Fi, Fi)] - W.T @ W
    buf = model.model.cpu().numpy()
    S0d = buf[:60 * 61].reshape(60, 61)[:, :60]
    pf = O.prefix_factor(TNTn, dn, gw, np.full(m - 60, 1e-40))
    print(f"S0 rel err: device {rel(S0d, S0x):.2e}  numpy {rel(pf['S0'], S0x):.2e}   |A_FF|/|S0| = "
          f"{float(np.max(np.abs(tl[np.ix_(Fi, Fi)])) / np.max(np.abs(S0x))):.2e}")
    rng = np.random.default_rng(0)
    order = O.chol_order(m, gw)
    errs_d, errs_n = [], []
    for _ in range(6):
        x = rng.uniform(-9, -4, 30)
        ph = O.phiinv_single(x, m - 60)
        z = np.zeros((1, model.ldb))
        z[0, :m] = rng.standard_normal(m)
        b, info = model.bdraw(torch.as_tensor(ph[None, :60], device=ctx.device), 1,
                              z=torch.as_tensor(z, device=ctx.device))
        bx = exact_chol_draw_pre((tl, dl), ph, z[0, :m], order)
        errs_d.append(normwise_rel(b.cpu().numpy()[0, :m], bx))
        errs_n.append(normwise_rel(O.bdraw_chol(TNTn, dn, ph, z[0, :m], order), bx))
    print("b draw rel err vs exact: device", " ".join(f"{e:.1e}" for e in errs_d))
    print("                         numpy ", " ".join(f"{e:.1e}" for e in errs_n))


if __name__ == "__main__":
    for a in sys.argv[1:]:
        main(int(a))
