"""CPU study: where does the fp64 b|rho draw lose accuracy, and what buys it back?

Emulates the device's tile algorithm (gibbs_tile.h / gibbs_big.hip: fixed-prior prefix, upper
Cholesky of the augmented Schur block on 16x16 tiles, explicit diagonal-tile inverses from
column elimination, TRSM and backward solve through them) in numpy fp64, next to LAPACK and
variants, and measures each against the x87 long-double Cholesky draw with the same normals
(tests/parity_data.exact_chol_draw_pre).  Usage: python tools/accuracy_sim.py [c5|j1713|psr32]
"""
import os
import sys

import numpy as np
import scipy.linalg as sl

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import gibbs_oracle as O  # noqa: E402
from tests.parity_data import exact_chol_draw_pre, exact_tnt, normwise_rel  # noqa: E402

L_ = np.longdouble


def col_elim(A, kmax=None):
    """Column elimination on a symmetric tile (tile_elim1<KMAX>): steps k < kmax - 1, E unit
    upper with A E lower on the first kmax columns; pivots of columns >= kmax are 1."""
    A = A.copy()
    n = A.shape[0]
    kmax = n if kmax is None else kmax
    E = np.eye(n)
    for k in range(kmax - 1):
        g = -A[k, k + 1:] / A[k, k]
        A[:, k + 1:] += np.outer(A[:, k], g)
        E[:, k + 1:] += np.outer(E[:, k], g)
    piv = np.diag(A).copy()
    piv[kmax:] = 1.0
    return A, E, piv


def tile_draw(S, dF, zF, mode="inv", ts=16):
    """x_F = U^-1 (U^-T dF + zF), S = U^T U upper, on ts-tiles (augmented dF column)."""
    nf = S.shape[0]
    NT = nf // ts + 1
    n = NT * ts
    A = np.eye(n)
    A[:nf, :nf] = S
    A[:nf, nf] = dF
    A[nf, :nf] = dF
    U = np.zeros((n, n))
    V = {}
    for K in range(NT):
        k0, k1 = K * ts, (K + 1) * ts
        T = A[k0:k1, k0:k1]
        cp = nf - k0 if K == NT - 1 else ts
        Ael, E, piv = col_elim(T, cp)
        rs = 1.0 / np.sqrt(piv)
        Vk = E * rs[None, :]               # U_KK^-1
        Ukk_T = Ael * rs[None, :]          # U_KK^T (lower)
        V[K] = Vk
        U[k0:k1, k0:k1] = Ukk_T.T
        if K == NT - 1:  # y of the last tile row: row cp of the eliminated tile
            U[k0:k0 + cp, nf] = Ael[cp, :cp] * rs[:cp]
        for J in range(K + 1, NT):
            j0, j1 = J * ts, (J + 1) * ts
            if mode in ("inv", "inv_bsub"):
                U[k0:k1, j0:j1] = Vk.T @ A[k0:k1, j0:j1]
            else:
                U[k0:k1, j0:j1] = sl.solve_triangular(Ukk_T, A[k0:k1, j0:j1], lower=True)
        for I in range(K + 1, NT):
            i0, i1 = I * ts, (I + 1) * ts
            for J in range(I, NT):
                j0, j1 = J * ts, (J + 1) * ts
                A[i0:i1, j0:j1] -= U[k0:k1, i0:i1].T @ U[k0:k1, j0:j1]
    # y: column nf of U (rows < nf) -- the augmented factorisation
    y = U[:nf, nf].copy()
    w = np.zeros(n)
    w[:nf] = y + zF
    x = np.zeros(n)
    for K in range(NT - 1, -1, -1):
        k0, k1 = K * ts, (K + 1) * ts
        r = w[k0:k1] - U[k0:k1, k1:] @ x[k1:]
        if mode == "inv":
            x[k0:k1] = V[K] @ r
        else:
            x[k0:k1] = sl.solve_triangular(U[k0:k1, k0:k1], r, lower=False)
        if K == NT - 1:
            x[nf:] = 0.0
    return x[:nf], U[:nf, :nf]


def prefix(TNT, d, gwid, phfix, dt=np.float64):
    m = TNT.shape[0]
    order = O.chol_order(m, gwid)
    nF = len(gwid)
    Mi, Fi = order[: m - nF], order[m - nF:]
    if dt is np.float64 and np.asarray(TNT).dtype == np.float64:
        return O.prefix_factor(TNT, d, gwid, phfix)
    T = np.asarray(TNT, dt)
    dv = np.asarray(d, dt)
    AMM = T[np.ix_(Mi, Mi)] + np.diag(np.asarray(phfix, dt))
    nm = len(Mi)
    LM = np.zeros_like(AMM)
    for k in range(nm):
        v = AMM[k:, k] - LM[k:, :k] @ LM[k, :k]
        LM[k, k] = np.sqrt(v[0])
        LM[k + 1:, k] = v[1:] / LM[k, k]

    def fsub(L, B):
        B = np.array(B, dt)
        X = np.zeros_like(B)
        for k in range(L.shape[0]):
            X[k] = (B[k] - L[k, :k] @ X[:k]) / L[k, k]
        return X
    W = fsub(LM, T[np.ix_(Mi, Fi)])
    e = fsub(LM, dv[Mi])
    S0 = T[np.ix_(Fi, Fi)] - W.T @ W
    dF = dv[Fi] - W.T @ e
    if os.environ.get("FP64_GHR"):  # R, G, h in fp64 from the rounded L_M and W (the device)
        LMd = np.asarray(LM, np.float64)
        R = sl.solve_triangular(LMd.T, np.eye(nm), lower=False)
        G = R @ np.asarray(W, np.float64)
        h = R @ np.asarray(e, np.float64)
    else:
        R = fsub(LM, np.eye(nm, dtype=dt)).T  # L_M^-T
        G = R @ W
        h = R @ e
    f = lambda a: np.asarray(a, np.float64)  # noqa: E731
    return dict(S0=f(S0), dF=f(dF), G=f(G), h=f(h), R=f(R), Mi=Mi, Fi=Fi)


def assemble(pf, xF, zc):
    zM = zc[pf["Mi"]]
    xM = pf["h"] + pf["R"] @ zM - pf["G"] @ xF
    b = np.empty(len(pf["Fi"]) + len(pf["Mi"]))
    b[pf["Fi"]] = xF
    b[pf["Mi"]] = xM
    return b


def corrected(S, U, dF, zF, twosum_ld=True):
    """First-order factor correction: U_exact^-1 z ~= U^-1 (z + Phi(M) z), M = U^-T (U^T U - S) U^-1,
    Phi = strict upper + diag/2; the residual in long double.  Mean by one refinement step."""
    Ul = np.asarray(U, L_)
    E = np.asarray(Ul.T @ Ul - np.asarray(S, L_), np.float64)
    Ui = sl.solve_triangular(U, np.eye(U.shape[0]), lower=False)
    M = Ui.T @ E @ Ui
    Ph = np.triu(M, 1) + np.diag(np.diag(M)) / 2
    w = zF + Ph @ zF
    # mean with one refinement step (residual in long double)
    mu = sl.solve_triangular(U, sl.solve_triangular(U.T, dF, lower=True), lower=False)
    r = np.asarray(np.asarray(dF, L_) - np.asarray(S, L_) @ np.asarray(mu, L_), np.float64)
    mu = mu + sl.solve_triangular(U, sl.solve_triangular(U.T, r, lower=True), lower=False)
    return mu + sl.solve_triangular(U, w, lower=False)


def systems(which, n_state=int(os.environ.get('NSTATE', 6)), seed=5):
    from pulsar_timing_gibbsspec_amd import synthetic
    rng = np.random.default_rng(seed)
    if which == "c5":
        d = synthetic.config5_array(n_psr=1, n_toa=10000, n_f=100, seed=21)
        T, r, N = d["T"][0], d["r"][0], d["sigma"][0] ** 2
        fidx = np.asarray(d["fidx"])
        phfix = d["phiinv_fixed"]
        lo, hi, nf = -8.5, -5.0, 100
    else:
        from tests.conftest import golden
        from tests.parity_data import indep_pick
        if which.startswith("arr"):  # pulsar P of the synthetic configs[2] array, random states
            p = synthetic.pulsar_ptas(synthetic.array_pta(kind="indep", seed=0))[int(which[3:])]
            T, N, r = p.get_basis()[0], p.get_ndiag({})[0], p.get_residuals()[0]
            fidx = np.arange(60)
            phfix = np.full(T.shape[1] - 60, 1e-40)
            lo, hi, nf = -9.0, -4.0, 30
        else:
            if which == "j1713":
                g = golden("single_j1713.npz")
            else:  # pickK: fixture pulsar K of configs[2], states from the reference's chain
                ga = golden("indep_array.npz")
                print("pulsar", int(ga["picks"][int(which[4:])]))
                g = indep_pick(ga, int(which[4:]))
            T, r, N = g["T"], g["r"], g["Nvec"]
            fidx = np.asarray(g["gwid"])
            m = T.shape[1]
            phfix = np.full(m - fidx.size, 1e-40)
            ch = g["chain"]
            lo, hi, nf = None, None, fidx.size // 2
    m = T.shape[1]
    out = []
    for k in range(n_state):
        if lo is not None:
            lr = rng.uniform(lo, hi, nf)
        else:
            lr = ch[rng.integers(0, ch.shape[0])][:nf]
        ph = 1.0 / np.repeat(10 ** (2 * lr), 2)
        phi = np.full(m, 1e-40)
        phi[fidx] = ph
        out.append((ph, phi, rng.standard_normal(m)))
    return T, r, N, fidx, phfix, out


def main(which):
    T, r, N, fidx, phfix, states = systems(which)
    m = T.shape[1]
    order = O.chol_order(m, fidx)
    tl = exact_tnt(T, N, r)
    TNT = np.asarray(tl[0], np.float64)  # exact TNT rounded: isolates the draw
    dv = np.asarray(tl[1], np.float64)
    pf = prefix(TNT, dv, fidx, phfix)
    pfx = prefix(TNT, dv, fidx, phfix, dt=L_)
    pfxx = prefix(tl[0], tl[1], fidx, phfix, dt=L_)  # unrounded TNT, long-double prefix
    res = {}
    for ph, phi, z in states:
        bx = exact_chol_draw_pre(tl, phi, z, order)
        S = pf["S0"] + np.diag(ph)
        Sx = pfx["S0"] + np.diag(ph)
        zF = z[pf["Fi"]]
        row = {}
        row["exact_of_rounded_tnt"] = normwise_rel(
            exact_chol_draw_pre((np.asarray(TNT, L_), np.asarray(dv, L_)), phi, z, order), bx)
        row["numpy_full"] = normwise_rel(O.bdraw_chol(TNT, dv, phi, z, order), bx)
        row["prefix_lapack"] = normwise_rel(O.bdraw_prefix(pf, ph, z), bx)
        row["ldprefix_lapack"] = normwise_rel(O.bdraw_prefix(pfx, ph, z), bx)
        for mode in ("inv", "inv_bsub", "sub"):
            xF, U = tile_draw(S, pf["dF"], zF, mode)
            row["tile_" + mode] = normwise_rel(assemble(pf, xF, z), bx)
        xF, U = tile_draw(S, pf["dF"], zF, "inv")
        row["tile_inv+corr"] = normwise_rel(assemble(pf, corrected(S, U, pf["dF"], zF), z), bx)
        row["tile_inv+corr_ldpre"] = normwise_rel(assemble(pfx, corrected(Sx, U, pfx["dF"], zF), z), bx)
        xF, U = tile_draw(pfxx["S0"] + np.diag(ph), pfxx["dF"], zF, "inv")
        row["ldtnt_ldprefix_tile"] = normwise_rel(assemble(pfxx, xF, z), bx)
        Sj = np.diag(1 / np.sqrt(np.diag(S)))
        row["cond_S"] = np.linalg.cond(S)
        row["cond_scaled"] = np.linalg.cond(Sj @ S @ Sj)
        for k, v in row.items():
            res.setdefault(k, []).append(v)
    for k, v in res.items():
        print(f"{k:22s} max {max(v):.3g}  median {np.median(v):.3g}")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "c5")
