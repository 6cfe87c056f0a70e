"""CPU ORACLE for the free-spectrum Gibbs hot path — TEST INFRASTRUCTURE ONLY.

This module is a numpy restatement of the reference algorithm
(``/root/reference/pulsar_gibbs.py``, ``pta_gibbs.py``), used by ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg as the
CHECKER / CPU baseline.  The product path (``pulsar_timing_gibbsspec_amd``)
never imports it: there is no CPU fallback.

Parity pinning: every function here is checked against golden vectors produced
by running the reference itself in the build container
(``tests/golden/make_golden.py`` → ``tests/golden/*.npz``;
``tests/test_oracle_golden.py``).  The enterprise quantities (T, N, phiinv, r)
come from the repo's facade, so parity is pinned at the reference's own
boundary.

Each function cites the reference lines it restates.
"""
from __future__ import annotations

import numpy as np
import scipy.linalg as sl

LN10 = np.log(10.0)
NGRID = 1000


# ============================================================== TNT / d (a2)
def tnt(T, Nvec, r):
    """TNT = T^T N^-1 T, d = T^T N^-1 r  (pulsar_gibbs.py:500-502, pta_gibbs.py:523-526)."""
    TNT = np.dot(T.T, T / Nvec[:, None])
    d = np.dot(T.T, r / Nvec)
    return TNT, d


# ============================================================== b | rho (a1, a5)
def bdraw_svd(TNT, d, phiinv, z, fallback=False):
    """Reference draw: Sigma = TNT + diag(phiinv); SVD; b = mn + U S^-1/2 z
    (pulsar_gibbs.py:505-518; pta_gibbs.py:533-546).  The LinAlgError QR branch
    (:511-516) draws with the wrong covariance and is not restated for parity; with
    fallback=True (the CPU baseline's timing loop only, so a rare LAPACK non-convergence
    costs what it costs the reference instead of ending the run) it is followed as written:
    Sigi = R^-1 Q^T, mn = Sigi d, Li = U(Sigi) s(Sigi)^-1/2."""
    Sigma = TNT + np.diag(phiinv)
    try:
        u, s, _ = sl.svd(Sigma)
    except np.linalg.LinAlgError:
        if not fallback:
            raise
        Q, R = sl.qr(Sigma)
        Sigi = sl.solve(R, Q.T)
        u, s, _ = sl.svd(Sigi)
        return np.dot(Sigi, d) + np.dot(u * np.sqrt(1 / s), z)
    mn = np.dot(u, np.dot(u.T, d) / s)
    Li = u * np.sqrt(1 / s)
    return mn + np.dot(Li, z)


def chol_order(m, gwid):
    """Column order used by the device factorisation: fixed-prior columns (timing
    model, …) first, then the free-spectrum (gw) columns in gwid order."""
    gwid = np.asarray(gwid)
    mask = np.ones(m, bool)
    mask[gwid] = False
    return np.concatenate([np.nonzero(mask)[0], gwid])


def bdraw_chol(TNT, d, phiinv, zc, order):
    """Same law as bdraw_svd via Cholesky of the permuted Sigma:
    b[o] = L^-T (L^-1 d[o] + zc[o]), Sigma[o][:,o] = L L^T."""
    Sigma = TNT + np.diag(phiinv)
    Sp = Sigma[np.ix_(order, order)]
    L = np.linalg.cholesky(Sp)
    y = sl.solve_triangular(L, d[order], lower=True)
    x = sl.solve_triangular(L.T, y + zc[order], lower=False)
    b = np.empty_like(x)
    b[order] = x
    return b


def rotate_normals(TNT, phiinv, z_ref, order):
    """Map the reference's normals z (b - mn = U S^-1/2 z) to the Cholesky draw's
    coordinates: zc[o] = L^T (U S^-1/2 z)[o].  Q = L^T U S^-1/2 is orthogonal, so
    zc is again standard normal (SURVEY.md §7 'Exact-draw parity')."""
    Sigma = TNT + np.diag(phiinv)
    u, s, _ = sl.svd(Sigma)
    w = (u * np.sqrt(1 / s)) @ z_ref
    L = np.linalg.cholesky(Sigma[np.ix_(order, order)])
    zc = np.empty_like(w)
    zc[order] = L.T @ w[order]
    return zc


def prefix_factor(TNT, d, gwid, phiinv_fixed):
    """Fixed-prior prefix of the Cholesky (the device's per-model precompute).

    With order (M, F): Sigma = [[A_MM, A_MF], [A_FM, A_FF + D_F]], A_MM = TNT_MM + diag(phiinv_M)
    fixed across sweeps.  L = [[L_M, 0], [W^T, L_S]], W = L_M^-1 A_MF,
    L_S L_S^T = S0 + D_F with S0 = A_FF - W^T W.  Returns
    S0 (NF x NF), dF = d_F - W^T L_M^-1 d_M, G = L_M^-T W (NM x NF), h = L_M^-T L_M^-1 d_M,
    R = L_M^-T (NM x NM, upper), so that x_F = L_S^-T (L_S^-1 dF + z_F) and
    x_M = h + R z_M - G x_F.
    """
    m = TNT.shape[0]
    order = chol_order(m, gwid)
    nF = len(gwid)
    Mi, Fi = order[: m - nF], order[m - nF:]
    AMM = TNT[np.ix_(Mi, Mi)] + np.diag(phiinv_fixed)
    LM = np.linalg.cholesky(AMM)
    W = sl.solve_triangular(LM, TNT[np.ix_(Mi, Fi)], lower=True)
    e = sl.solve_triangular(LM, d[Mi], lower=True)
    S0 = TNT[np.ix_(Fi, Fi)] - W.T @ W
    dF = d[Fi] - W.T @ e
    R = sl.solve_triangular(LM.T, np.eye(len(Mi)), lower=False)
    G = R @ W
    h = R @ e
    return dict(S0=S0, dF=dF, G=G, h=h, R=R, Mi=Mi, Fi=Fi)


def bdraw_prefix(pf, phiinv_F, zc):
    """b|rho from the prefix factors (restates the device algorithm in numpy)."""
    L = np.linalg.cholesky(pf["S0"] + np.diag(phiinv_F))
    zF, zM = zc[pf["Fi"]], zc[pf["Mi"]]
    y = sl.solve_triangular(L, pf["dF"], lower=True)
    xF = sl.solve_triangular(L.T, y + zF, lower=False)
    xM = pf["h"] + pf["R"] @ zM - pf["G"] @ xF
    b = np.empty(len(pf["Fi"]) + len(pf["Mi"]))
    b[pf["Fi"]] = xF
    b[pf["Mi"]] = xM
    return b


# ============================================================== rho | b (a3, a4, a6, a7)
def tau_half(b, gwid):
    """tau_k = (b_sin^2 + b_cos^2)/2 (pulsar_gibbs.py:208-209)."""
    t = b[gwid] ** 2
    return (t[::2] + t[1::2]) / 2


def tau_full(b, gwid):
    """tau_k = b_sin^2 + b_cos^2, no /2 (pta_gibbs.py:194-195, 259-260)."""
    t = b[gwid] ** 2
    return t[::2] + t[1::2]


def rho_analytic(tau, U, rhomin, rhomax):
    """Truncated inverse-gamma(1) inverse-CDF draw (pulsar_gibbs.py:215-216).
    np.random.uniform(0, hi) == 0 + hi*U."""
    hi = 1 - np.exp((tau / rhomax) - (tau / rhomin))
    eta = 0.0 + hi * U
    return tau / ((tau / rhomax) - np.log(1 - eta))


def rho_grid(rhomin, rhomax, n=NGRID):
    """10**linspace(log10 rhomin, log10 rhomax, 1000) (pulsar_gibbs.py:228, pta_gibbs.py:189)."""
    return 10 ** np.linspace(np.log10(rhomin), np.log10(rhomax), n)


def rho_grid_gumbel(tau, irn, gumbel_u, rhomin, rhomax):
    """Grid + Gumbel-max draw with intrinsic red noise (pulsar_gibbs.py:223-234).
    gumbel_u are the U(0,1) samples behind np.random.gumbel (G = -log(-log(1-U)))."""
    rho_tmp = rho_grid(rhomin, rhomax)
    logratio = np.log(tau[:, None]) - np.logaddexp.outer(np.log(irn), np.log(rho_tmp))
    logpdf = logratio - np.exp(logratio)
    g = 0.0 - 1.0 * np.log(-np.log1p(-gumbel_u))
    idx = np.argmax(logpdf + g, axis=1)
    return rho_tmp[idx], idx


def _cdf_index(cdf, u):
    """searchsorted(cdf, u, 'left') - 1; -1 wraps to the last grid point."""
    return np.array([np.searchsorted(cdf[i, :], u[i], side="left") for i in range(u.shape[0])]) - 1


def rho_grid_cdf_curn(tau, irn, U, rhomin, rhomax):
    """Common free spectrum: product over pulsars of per-pulsar grid pdfs, CDF draw
    (pta_gibbs.py:189-212).  tau, irn: (P, n_f)."""
    rho_tmp = rho_grid(rhomin, rhomax)
    P, nf = tau.shape
    pdf = np.zeros((nf, rho_tmp.size, P))
    for ii in range(P):
        ratio = tau[ii][:, None] / np.add.outer(irn[ii], rho_tmp)
        pdf[:, :, ii] = ratio * np.exp(-ratio / 2) * np.log(10)
    pdf = np.prod(pdf, axis=2)
    cdf = np.cumsum(pdf, axis=1)
    cdf /= cdf.max(axis=1)[:, None]
    idx = _cdf_index(cdf, U)
    return np.take_along_axis(rho_tmp, idx, axis=0), idx


def rho_grid_cdf_curn_sum(S, n_psr, U, rhomin, rhomax):
    """The CURN grid-CDF draw without intrinsic red noise from the sufficient statistic
    S_k = sum_p tau_p,k (pta_gibbs.py:194-212 with irn = 0): prod_p ratio e^(-ratio/2)
    ln10 = const * rho^-P e^(-S/(2 rho)); the constant cancels in cdf / max.  Log space,
    relative to the row maximum.  S, U: (n_f,)."""
    rho_tmp = rho_grid(rhomin, rhomax)
    lp = -n_psr * np.log(rho_tmp)[None, :] - np.asarray(S)[:, None] / (2.0 * rho_tmp[None, :])
    pdf = np.exp(lp - lp.max(axis=1)[:, None])
    cdf = np.cumsum(pdf, axis=1)
    cdf /= cdf.max(axis=1)[:, None]
    idx = _cdf_index(cdf, U)
    return np.take_along_axis(rho_tmp, idx, axis=0), idx


def rho_grid_cdf_red(tau, gw, U, rhomin, rhomax):
    """Per-pulsar red free spectrum, grid CDF conditioned on the common phi_gw
    (pta_gibbs.py:254-276).  tau, U: (P, n_f); gw: (n_f,)."""
    rho_red = rho_grid(rhomin, rhomax)
    out, idxs = [], []
    for ii in range(tau.shape[0]):
        ratio = tau[ii][:, None] / np.add.outer(gw, rho_red)
        pdf = ratio * np.exp(-ratio / 2) * np.log(10)
        cdf = np.cumsum(pdf, axis=1)
        cdf /= cdf.max(axis=1)[:, None]
        idx = _cdf_index(cdf, U[ii])
        idxs.append(idx)
        out.append(np.take_along_axis(rho_red, idx, axis=0))
    return np.stack(out), np.stack(idxs)


# ============================================================== sweep loops (a8)
def phiinv_single(x_rho, n_tm):
    """phiinv of T = [F | M] for the single-pulsar notebook model
    (free spectrum phi = repeat(10**(2 log10 rho), 2); timing model phi = 1e40)."""
    return np.concatenate([1.0 / np.repeat(10.0 ** (2.0 * np.asarray(x_rho)), 2),
                           np.full(n_tm, 1.0 / 1e40)])


def sweep_single(TNT, d, gwid, x0, rhomin, rhomax, z_draws, U_draws, niter, phiinv_of_x,
                 draw="svd", order=None):
    """PulsarBlockGibbs.sample for the free-spectrum-only model (pulsar_gibbs.py:620-699):
    record-before-update, first b draw from xs, analytic rho|b, gate, b|rho.
    ``z_draws`` are consumed in order (first draw, then one per accepted gate),
    ``U_draws[ii]`` per sweep.  draw='svd' uses the reference map, 'chol' the
    Cholesky map with pre-rotated normals.  Returns chain, bchain, final b."""
    m = TNT.shape[0]
    gwind = np.arange(len(gwid) // 2)
    chain = np.zeros((niter, len(x0)))
    bchain = np.zeros((niter, m))
    b = np.zeros(m)
    xnew = np.asarray(x0, float)
    zi = 0

    def draw_b(x):
        nonlocal zi
        ph = phiinv_of_x(x)
        z = z_draws[zi]
        zi += 1
        if draw == "svd":
            return bdraw_svd(TNT, d, ph, z)
        return bdraw_chol(TNT, d, ph, z, order)

    for ii in range(niter):
        chain[ii] = xnew
        bchain[ii] = b
        if ii == 0:
            b = draw_b(x0)
        tau = tau_half(b, gwid)
        rho = rho_analytic(tau, U_draws[ii], rhomin, rhomax)
        x = xnew.copy()
        x[gwind] = 0.5 * np.log10(rho)
        xnew = x
        if np.all(xnew != chain[ii, -1]):
            b = draw_b(xnew)
    return chain, bchain, b


# ============================================================== likelihoods (a10, §8f-1)
def lnlike_white(r, T, b, Nvec):
    """-1/2 (sum log N + sum (r - T b)^2 / N)  (pulsar_gibbs.py:523-546)."""
    y = r - np.dot(T, b)
    return -0.5 * (np.sum(np.log(Nvec)) + np.sum(y ** 2 / Nvec))


def lnlike_fullmarg(r, Nvec, TNT, d, phiinv, logdet_phi):
    """Marginalised likelihood via Cholesky (pulsar_gibbs.py:569-610)."""
    ll = -0.5 * (np.sum(np.log(Nvec)) + np.sum(r ** 2 / Nvec))
    Sigma = TNT + np.diag(phiinv)
    try:
        cf = sl.cho_factor(Sigma)
        ev = sl.cho_solve(cf, d)
    except np.linalg.LinAlgError:
        return -np.inf
    logdet_sigma = np.sum(2 * np.log(np.diag(cf[0])))
    return ll + 0.5 * (np.dot(d, ev) - logdet_sigma - logdet_phi)


def lnlike_phi_batch(pf, phi_F, chunk=2048):
    """The phi-dependent part of one pulsar's marginalised likelihood (pta_gibbs.py:596-619, the
    term of pulsar ii in get_lnlikelihood) for a batch of free-spectrum phi rows phi_F (B x NF,
    the prefix_factor pf's F order), the fixed-prior columns' phi held fixed:
    1/2 (d^T Sigma^-1 d - log det Sigma - log det phi) = 1/2 (|L_S^-1 dF|^2 - log det(S0 + diag(1/phi_F))
    - sum log phi_F) + const, since log det Sigma = log det A_MM + log det(S0 + D_F) and
    d^T Sigma^-1 d = |L_M^-1 d_M|^2 + dF^T (S0 + D_F)^-1 dF.  The dropped constant (log det N, r^T N^-1 r,
    the A_MM terms, the timing-model phi) does not depend on phi_F.  -inf where S0 + D_F is not PD."""
    phi_F = np.atleast_2d(np.asarray(phi_F, float))
    S0, dF = pf["S0"], pf["dF"]
    nF = S0.shape[0]
    out = np.empty(phi_F.shape[0])
    for a in range(0, phi_F.shape[0], chunk):
        ph = phi_F[a:a + chunk]
        S = np.broadcast_to(S0, (ph.shape[0], nF, nF)).copy()
        S[:, np.arange(nF), np.arange(nF)] += 1.0 / ph
        try:
            L = np.linalg.cholesky(S)
        except np.linalg.LinAlgError:           # some row is not PD: row by row
            out[a:a + chunk] = ([lnlike_phi_batch(pf, r[None])[0] for r in ph] if ph.shape[0] > 1
                                else -np.inf)
            continue
        y = np.empty((ph.shape[0], nF))
        for i in range(nF):                     # forward substitution, vectorised over the batch
            y[:, i] = (dF[i] - np.einsum("bj,bj->b", L[:, i, :i], y[:, :i])) / L[:, i, i]
        ld = 2.0 * np.sum(np.log(L[:, np.arange(nF), np.arange(nF)]), axis=1)
        out[a:a + chunk] = 0.5 * (np.sum(y * y, axis=1) - ld - np.sum(np.log(ph), axis=1))
    return out


# ============================================================== Philox4x32-10 (a9)
PHILOX_M0, PHILOX_M1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
PHILOX_W0, PHILOX_W1 = np.uint32(0x9E3779B9), np.uint32(0xBB67AE85)
_M32 = np.uint64(0xFFFFFFFF)


def philox4x32(ctr, key, rounds=10):
    """Philox4x32-10 (Salmon et al. 2011).  ctr: (...,4) uint32, key: (...,2) uint32."""
    c = [np.asarray(ctr[..., i], np.uint64) for i in range(4)]
    k0 = np.asarray(key[..., 0], np.uint64)
    k1 = np.asarray(key[..., 1], np.uint64)
    for r in range(rounds):
        if r > 0:   # 32-bit wrap-around of the key bumps, in 64-bit arithmetic (no overflow warning)
            k0 = (k0 + np.uint64(PHILOX_W0)) & _M32
            k1 = (k1 + np.uint64(PHILOX_W1)) & _M32
        p0 = PHILOX_M0 * c[0]
        p1 = PHILOX_M1 * c[2]
        hi0, lo0 = p0 >> np.uint64(32), p0 & _M32
        hi1, lo1 = p1 >> np.uint64(32), p1 & _M32
        c = [hi1 ^ c[1] ^ k0, lo1, hi0 ^ c[3] ^ k1, lo0]
    return np.stack([x.astype(np.uint32) for x in c], axis=-1)


def u53(hi, lo):
    """Two 32-bit words -> double in [0,1) with 53 random bits."""
    v = (hi.astype(np.uint64) << np.uint64(32)) | lo.astype(np.uint64)
    return (v >> np.uint64(11)).astype(np.float64) * (1.0 / 9007199254740992.0)


def philox_uniform_pair(ctr, key):
    w = philox4x32(ctr, key)
    return u53(w[..., 0], w[..., 1]), u53(w[..., 2], w[..., 3])


def box_muller(u1, u2):
    r = np.sqrt(-2.0 * np.log(1.0 - u1))
    t = 2.0 * np.pi * u2
    return r * np.cos(t), r * np.sin(t)


# ============================================================== ESS (metric)
def iat(x, c=5.0):
    """Integrated autocorrelation time, Sokal's adaptive window (M >= c tau)."""
    x = np.asarray(x, float) - np.mean(x)
    n = x.size
    f = np.fft.rfft(x, 2 * n)
    acf = np.fft.irfft(f * np.conj(f))[:n]
    if acf[0] <= 0:
        return 1.0
    acf /= acf[0]
    tau = 2.0 * np.cumsum(acf) - 1.0
    for M in range(1, n):
        if M >= c * tau[M]:
            return float(tau[M])
    return float(tau[-1])


# ============================================================== white-noise MH (a10)
MH_SIZES = [0.1, 0.5, 1.0, 3.0, 10.0]
MH_PROBS = [0.1, 0.15, 0.5, 0.15, 0.1]


def ndiag_white(sigma, backends, ef, eq_log10):
    """N = efac^2 sigma^2 + 10**(2 log10_tnequad) per backend (the facade's get_ndiag;
    the per-backend power is a Python-float pow there, kept so here bit-for-bit)."""
    eq = np.array([10.0 ** (2.0 * float(v)) for v in eq_log10])
    return np.asarray(ef, float)[backends] ** 2 * sigma ** 2 + eq[backends]


def white_mh(x, wind, steps, lnlike, lnprior):
    """Steady-state white-noise Metropolis block (pulsar_gibbs.py:373-404).
    steps: iterable of (scale, par, z, u) = the values of np.random.choice(sizes, p=probs),
    np.random.choice(wind), np.random.randn(1), np.random.rand() for each step.
    The jump is q[par] += z * (0.05 * len(wind)) * scale (:383); accept if
    (lnlike1 + lnprior1) - (lnlike0 + lnprior0) > log(u) (:398)."""
    xnew = np.asarray(x, float).copy()
    l0, p0 = lnlike(xnew), lnprior(xnew)
    for scale, par, z, u in steps:
        q = xnew.copy()
        sigmas = 0.05 * len(wind)
        q[int(par)] += z * sigmas * scale
        l1, p1 = lnlike(q), lnprior(q)
        diff = (l1 + p1) - (l0 + p0)
        if diff > np.log(u):
            xnew, l0, p0 = q, l1, p1
    return xnew


# ============================================================== power-law red MH
EV_REDMH = 8


def lnlike_red(b, gwid, irn, gwphi):
    """get_lnlikelihood_red (pulsar_gibbs.py:549-566): tau = (b_sin^2 + b_cos^2)/2,
    lr = log tau - logaddexp(log irn, log phi_gw), lnL = sum(lr - exp(lr))."""
    tau = np.asarray(b)[gwid] ** 2
    tau = (tau[::2] + tau[1::2]) / 2
    logratio = np.log(tau) - np.logaddexp(np.log(irn), np.log(gwphi))
    return np.sum(logratio - np.exp(logratio))


def powerlaw_lnirn(lnphi, la, ga):
    """log irn_k = (a_k la + c_k) + g_k ga: the power law's log-linear form (lnphi rows c, a, g)."""
    return (lnphi[1] * la + lnphi[0]) + lnphi[2] * ga


def red_mh_philox(x, ia, ig, gw_col, tau_half, lnphi, jump, de, nsteps, anchor, key, sweep, chain):
    """The device red-noise Metropolis block (gs_red_mh) restated on the same Philox
    stream.  Steady state of update_red_params (pulsar_gibbs.py:312-319): nsteps symmetric
    jumps (SCAM / AM / DE mix restating PTMCMCSampler's, which is absent — parity of the
    proposal law unpinned), each accepted if lnL(q) - lnL(ref) > log u with ref = the
    block's starting point when anchor (the reference discards PTMCMCOneStep's returned
    state, :318-319) or the current one.  Returns (x, lnL, n_acc, margins) where
    margins[s] = |lnL(q) - lnL(ref) - log u| of each step (near-ties, for tests)."""
    x = np.asarray(x, float).copy()
    ltau = np.log(np.asarray(tau_half, float))
    lgw = np.log(10.0 ** (2.0 * x[gw_col]))

    def L(a, g):
        lr = ltau - np.logaddexp(powerlaw_lnirn(lnphi, a, g), lgw)
        return float(np.sum(lr - np.exp(lr)))

    U00, U01, U10, U11, s0, s1, w_scam, w_am, lo0, hi0, lo1, hi1 = [float(v) for v in jump]
    qa, qg = float(x[ia]), float(x[ig])
    L0 = Lc = L(qa, qg)
    acc, margins = 0, []
    key = np.asarray(key, np.uint32)

    def uni(slot):
        ctr = np.array([slot, sweep & 0xffffffff, chain & 0xffffffff, EV_REDMH], np.uint32)
        u1, u2 = philox_uniform_pair(ctr, key)
        return float(u1), float(u2)

    for s in range(nsteps):
        u_kind, u_scale = uni(4 * s)
        u_a, u_b = uni(4 * s + 1)
        n1, n2 = (float(v) for v in box_muller(*uni(4 * s + 2)))
        u_acc, u_de = uni(4 * s + 3)
        scale = 10.0 if u_scale > 0.97 else (0.2 if u_scale > 0.9 else 1.0)
        if u_kind < w_scam:
            d1 = u_a >= 0.5
            cd = 1.6970562748477141 * scale * (s1 if d1 else s0) * n1
            da, dg = cd * (U01 if d1 else U00), cd * (U11 if d1 else U10)
        elif u_kind < w_am:
            cd = 1.2 * scale
            z0, z1 = n1 * s0, n2 * s1
            da, dg = cd * (U00 * z0 + U01 * z1), cd * (U10 * z0 + U11 * z1)
        else:
            n = len(de)
            i = min(int(u_a * n), n - 1)
            k = min(int(u_b * (n - 1)), n - 2)
            k += k >= i
            sc = 1.0 if u_de < 0.5 else u_scale * 1.2
            da, dg = sc * (de[i][0] - de[k][0]), sc * (de[i][1] - de[k][1])
        pa, pg = qa + da, qg + dg
        inb = lo0 <= pa <= hi0 and lo1 <= pg <= hi1
        L1 = L(pa, pg) if inb else -np.inf
        ref = L0 if anchor else Lc
        diff = L1 - ref
        margins.append(abs(diff - np.log(u_acc)) if np.isfinite(diff) else np.inf)
        if diff > np.log(u_acc):
            qa, qg, Lc = pa, pg, L1
            acc += 1
    x[ia], x[ig] = qa, qg
    return x, Lc, acc, np.array(margins)


# ============================================================== basis ECORR
def ecorr_schur(TNT, d, ecid, phi_E):
    """Eliminate the ECORR epoch columns (ecid) of Sigma = TNT + diag(phiinv) first.
    U^T N^-1 U is diagonal (each TOA sits in at most one epoch), so with
    a_e = TNT_ee + 1/phi_e, B = TNT[ecid, R] and R the remaining columns in order:
        Sigma_R' = TNT_RR - B^T diag(1/a) B,   d_R' = d_R - B^T (d_E / a)
    and log det Sigma = sum log a + log det(Sigma_R' + diag(phiinv_R)),
    d^T Sigma^-1 d = sum d_E^2 / a + d_R'^T (Sigma_R' + diag(phiinv_R))^-1 d_R'.
    Restates, in block form, the Sigma of get_lnlikelihood_fullmarg (pulsar_gibbs.py:592)
    and update_b (:505) with the ECORR phiinv of get_phiinv.  Returns
    (rcols, TNT_R', d_R', sum log a, sum d_E^2 / a)."""
    m = TNT.shape[0]
    ecid = np.asarray(ecid)
    rc = np.setdiff1d(np.arange(m), ecid)
    a = np.diag(TNT)[ecid] + 1.0 / np.asarray(phi_E, float)
    B = TNT[np.ix_(ecid, rc)]
    dE = d[ecid]
    S = TNT[np.ix_(rc, rc)] - B.T @ (B / a[:, None])
    dR = d[rc] - B.T @ (dE / a)
    return rc, S, dR, float(np.sum(np.log(a))), float(np.sum(dE ** 2 / a))


def lnlike_ecorr_marg(r, Nvec, TNT, d, ecid, phiinv, logdet_phi):
    """get_lnlikelihood_fullmarg (pulsar_gibbs.py:569-610) through ecorr_schur: equal to
    lnlike_fullmarg up to rounding (the ECORR block is diagonal)."""
    ll = -0.5 * (np.sum(np.log(Nvec)) + np.sum(r ** 2 / Nvec))
    rc, S, dR, sla, sdw = ecorr_schur(TNT, d, ecid, 1.0 / phiinv[ecid])
    try:
        cf = sl.cho_factor(S + np.diag(phiinv[rc]))
    except np.linalg.LinAlgError:
        return -np.inf
    ev = sl.cho_solve(cf, dR)
    ld = sla + np.sum(2 * np.log(np.diag(cf[0])))
    return ll + 0.5 * (sdw + np.dot(dR, ev) - ld - logdet_phi)


def bdraw_ecorr(TNT, d, ecid, phiinv, zR, zE):
    """b | rho with the ECORR block eliminated first: b_R ~ N(S^-1 d_R', S^-1) drawn as
    S^-1 d_R' + L^-T zR (S = Sigma_R' + diag(phiinv_R) = L L^T), then the epochs
    b_E | b_R ~ N((d_E - B b_R) / a, 1/a) = (d_E - B b_R)/a + zE / sqrt(a).  Same
    distribution as update_b (pulsar_gibbs.py:489-520); returns b in original column order."""
    m = TNT.shape[0]
    ecid = np.asarray(ecid)
    rc, S, dR, _, _ = ecorr_schur(TNT, d, ecid, 1.0 / phiinv[ecid])
    L = np.linalg.cholesky(S + np.diag(phiinv[rc]))
    bR = sl.cho_solve((L, True), dR) + sl.solve_triangular(L.T, zR, lower=False)
    a = np.diag(TNT)[ecid] + phiinv[ecid]
    bE = (d[ecid] - TNT[np.ix_(ecid, rc)] @ bR) / a + zE / np.sqrt(a)
    b = np.empty(m)
    b[rc], b[ecid] = bR, bE
    return b
