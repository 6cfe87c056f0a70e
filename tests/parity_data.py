"""Replay inputs built from the golden fixtures (shared by CPU and GPU tests).

The reference draws b = mn + U S^-1/2 z (pulsar_gibbs.py:508-518).  The HIP
path draws b = mn + L^-T z' with L the Cholesky factor of Sigma in the device
column order (fixed-prior columns first, then gwid).  For exact-draw parity
the reference's normals are rotated, z' = L^T U S^-1/2 z, using Sigma along
the REFERENCE trajectory (tests/golden/single_j1713.npz).
"""
import numpy as np

from oracle import gibbs_oracle as O


def single_replay(g):
    """-> dict with TNT, d, gwid, order, n_tm, per-draw phiinv and rotated normals.

    Draw k of the reference run: k = 0 at x0 (first draw, pulsar_gibbs.py:661-662),
    k = ii + 1 at the state after sweep ii (= chain[ii + 1], or the final state
    for the last sweep; every gate passes in the analytic branch)."""
    TNT, d = O.tnt(g["T"], g["Nvec"], g["r"])
    m = TNT.shape[0]
    gwid = np.asarray(g["gwid"])
    n_tm = m - gwid.size
    order = O.chol_order(m, gwid)
    chain = g["chain"]
    niter = chain.shape[0]
    # state after the last sweep: rho draw from the final b is not in the chain;
    # recompute it exactly as the reference (same U, same b) to get x_final.
    b_last = g["bchain"][-1] if niter > 1 else None
    tau = O.tau_half(b_last, gwid)
    rho = O.rho_analytic(tau, g["U"][-1], float(g["rhomin"]), float(g["rhomax"]))
    x_final = 0.5 * np.log10(rho)
    xs = [g["x0"]] + [chain[i + 1] for i in range(niter - 1)] + [x_final]
    ph = [O.phiinv_single(x, n_tm) for x in xs]
    zc = np.stack([O.rotate_normals(TNT, ph[k], g["z"][k], order) for k in range(len(xs))])
    return dict(TNT=TNT, d=d, gwid=gwid, order=order, n_tm=n_tm, xs=xs, phiinv=ph, zc=zc,
                niter=niter, rhomin=float(g["rhomin"]), rhomax=float(g["rhomax"]))


def normwise_rel(a, b, axis=-1):
    """max over rows of |a - b|_inf / |b|_inf (per row)."""
    a, b = np.asarray(a), np.asarray(b)
    num = np.max(np.abs(a - b), axis=axis)
    den = np.maximum(np.max(np.abs(b), axis=axis), 1e-300)
    return float(np.max(num / den))
