"""CPU baseline loops for bench.py's ``cpu_baseline`` leg -- TEST/MEASUREMENT INFRASTRUCTURE.

Each loop is the oracle's restatement of the reference sampler's per-sweep work for one
BASELINE configuration (numpy/LAPACK, the reference's own operation order: TNT
recomputed every sweep as pulsar_gibbs.py:664-665 forces, SVD b draw :505-518, the rho
draws of :206-236 / pta_gibbs.py:181-276), run single-threaded for a bounded time.
``aggregate`` runs one such process per host core at once (OPENBLAS_NUM_THREADS=1, the
way the reference is fastest on a multi-core host: SURVEY.md §6, Appendix A.10) and sums
their rates: the whole-host CPU throughput the GPU is compared with.

Processes are started as ``python -m oracle.cpu_baseline KIND SECONDS`` so that they
import numpy only (never torch, never the GPU).  The product path never imports this
module.
"""
from __future__ import annotations

import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bdraw_fast(TNT, d, phiinv, z, fallback=True):
    """The ESS runs' b|rho draw: the same N(Sigma^-1 d, Sigma^-1) law as bdraw_svd (pulsar_gibbs.py:505-518)
    through a Jacobi-scaled Cholesky, Sigma = D^-1/2 L L^T D^-1/2: b = D^1/2 L^-T (L^-1 D^1/2 d + z).  The
    chain's law, hence its ESS per sweep, is the reference's; the SVD stays in the throughput loop."""
    import numpy as np
    import scipy.linalg as sl
    from oracle import gibbs_oracle as O
    Sigma = TNT + np.diag(phiinv)
    s = 1.0 / np.sqrt(np.diag(Sigma))
    try:
        L = np.linalg.cholesky(Sigma * s[:, None] * s[None, :])
    except np.linalg.LinAlgError:
        return O.bdraw_svd(TNT, d, phiinv, z, fallback=fallback)
    y = sl.solve_triangular(L, d * s, lower=True)
    return s * sl.solve_triangular(L.T, y + z, lower=False)


def _curn_fast(taus, irn, U, rhomin=1e-18, rhomax=1e-8):
    """The ESS runs' common-rho grid draw: the CDF of rho_grid_cdf_curn (pta_gibbs.py:189-212) in log space,
    log pdf_g = -sum_p [log(irn_p + rho_g) + tau_p / (2 (irn_p + rho_g))] + const (the constant, sum_p log tau_p
    + P log ln10, cancels in cdf / max), the logs taken once per 8 pulsars' product.  Same CDF, same
    searchsorted - 1 index rule; a fifth of the transcendentals."""
    import numpy as np
    from oracle import gibbs_oracle as O
    g = O.rho_grid(rhomin, rhomax)
    P = taus.shape[0]
    lp = np.zeros((taus.shape[1], g.size))
    for a in range(0, P, 8):
        prod = np.ones_like(lp)
        for p in range(a, min(P, a + 8)):
            den = irn[p][:, None] + g[None, :]
            prod *= den
            lp -= 0.5 * taus[p][:, None] / den
        lp -= np.log(prod)
    pdf = np.exp(lp - lp.max(axis=1)[:, None])
    cdf = np.cumsum(pdf, axis=1)
    cdf /= cdf.max(axis=1)[:, None]
    idx = O._cdf_index(cdf, U)
    return np.take_along_axis(g, idx, axis=0), idx


def _red_fast(taus, gw, U, rhomin=1e-20, rhomax=1e-8):
    """The ESS runs' per-pulsar red grid draw: rho_grid_cdf_red (pta_gibbs.py:254-276) vectorised over
    the pulsars, the same arithmetic per grid point; searchsorted(cdf, u, 'left') - 1 as the count of
    cdf entries below u, minus one (cdf is nondecreasing)."""
    import numpy as np
    from oracle import gibbs_oracle as O
    g = O.rho_grid(rhomin, rhomax)
    ratio = taus[:, :, None] / (gw[None, :, None] + g[None, None, :])
    cdf = np.cumsum(ratio * np.exp(-ratio / 2) * np.log(10), axis=2)
    cdf /= cdf.max(axis=2)[:, :, None]
    idx = (cdf < U[:, :, None]).sum(axis=2) - 1
    idx[idx < 0] += g.size
    return g[idx], idx


def _loop(step, seconds):
    it, t0 = 0, time.perf_counter()
    while True:
        step()
        it += 1
        el = time.perf_counter() - t0
        if el > seconds:
            return it, el


def single(fast=False):
    """configs[0]/[1]: J1713 single chain (PulsarBlockGibbs.sample, pulsar_gibbs.py:656-698).
    ``fast`` (the ESS runs only): TNT/d computed once -- N is fixed, so the chain's law is the
    same and only the throughput leg must pay for the reference's recompute."""
    import numpy as np
    from oracle import gibbs_oracle as O
    from pulsar_timing_gibbsspec_amd import synthetic
    pta = synthetic.single_pulsar_pta("J1713+0747", seed=0)
    T, N, r = pta.get_basis()[0], pta.get_ndiag({})[0], pta.get_residuals()[0]
    gwid = np.arange(60)
    rng = np.random.default_rng(os.getpid())
    n_tm = T.shape[1] - 60
    st = dict(x=rng.uniform(-9, -4, 30), b=None)

    TD0 = O.tnt(T, N, r) if fast else None
    bd = _bdraw_fast if fast else O.bdraw_svd

    def step():
        TNT, d = TD0 or O.tnt(T, N, r)                       # recomputed every sweep (:664-665)
        if st["b"] is None:                                  # first draw from xs (:661-662)
            st["b"] = bd(TNT, d, O.phiinv_single(st["x"], n_tm), rng.standard_normal(T.shape[1]), fallback=True)
        tau = O.tau_half(st["b"], gwid)
        st["x"] = 0.5 * np.log10(O.rho_analytic(tau, rng.random(30), 1e-18, 1e-8))
        st["b"] = bd(TNT, d, O.phiinv_single(st["x"], n_tm), rng.standard_normal(T.shape[1]), fallback=True)
    return step, lambda: st["x"], "J1713 single-chain sweeps (oracle restatement of pulsar_gibbs.py:656-698)"


def indep(fast=False):
    """configs[2]: one sweep of every one of the 45 pulsars' PulsarBlockGibbs loops (each
    pulsar its own free spectrum, pulsar_gibbs.py:656-698) = one array sweep (``fast``: TNT once)."""
    import numpy as np
    from oracle import gibbs_oracle as O
    from pulsar_timing_gibbsspec_amd import synthetic
    ptas = synthetic.pulsar_ptas(synthetic.array_pta(kind="indep", seed=0))
    data = [(p.get_basis()[0], p.get_ndiag({})[0], p.get_residuals()[0]) for p in ptas]
    rng = np.random.default_rng(os.getpid())
    xs = [rng.uniform(-9, -4, 30) for _ in data]
    bs = [None] * len(data)
    gwid = np.arange(60)
    TD = [O.tnt(T, N, r) for T, N, r in data] if fast else None
    bd = _bdraw_fast if fast else O.bdraw_svd

    def step():
        for p, (T, N, r) in enumerate(data):
            m = T.shape[1]
            TNT, d = TD[p] if fast else O.tnt(T, N, r)
            if bs[p] is None:
                bs[p] = bd(TNT, d, O.phiinv_single(xs[p], m - 60), rng.standard_normal(m), fallback=True)
            xs[p] = 0.5 * np.log10(O.rho_analytic(O.tau_half(bs[p], gwid), rng.random(30), 1e-18, 1e-8))
            bs[p] = bd(TNT, d, O.phiinv_single(xs[p], m - 60), rng.standard_normal(m), fallback=True)
    return step, lambda: np.concatenate(xs), "45-pulsar array sweeps (each pulsar's PulsarBlockGibbs loop, pulsar_gibbs.py:656-698)"


def pta(kind, fast=False):
    """configs[3]: PTABlockGibbs.sample (pta_gibbs.py:664-704), SVD draws, 45 pulsars
    (``fast``: TNT once)."""
    import numpy as np
    from oracle import gibbs_oracle as O
    from pulsar_timing_gibbsspec_amd import synthetic
    p_ = synthetic.array_pta(kind=kind, seed=0)
    T, N, R = p_.get_basis(), p_.get_ndiag({}), p_.get_residuals()
    P = len(T)
    names = p_.param_names
    rind = np.array([i for i, n in enumerate(names) if "rho" in n and "gw" in n])
    hind = np.array([i for i, n in enumerate(names) if "red" in n and "rho" in n])
    rng = np.random.default_rng(os.getpid())
    st = dict(x=rng.uniform(-9, -4, len(names)))
    m = [t.shape[1] for t in T]
    gw = [np.arange(mm - 60, mm) for mm in m]

    TD = [O.tnt(T[p], N[p], R[p]) for p in range(P)] if fast else None
    bd = _bdraw_fast if fast else O.bdraw_svd

    def draw(x):
        out = []
        for p in range(P):
            TNT, d = TD[p] if fast else O.tnt(T[p], N[p], R[p])   # reset + recompute (pta_gibbs.py:672-673)
            phi = 10 ** (2 * x[rind]) + (10 ** (2 * x[hind[p * 30:(p + 1) * 30]]) if kind == "curn_red" else 0)
            ph = np.full(m[p], 1e-40)
            ph[gw[p]] = 1 / np.repeat(phi, 2)
            out.append(bd(TNT, d, ph, rng.standard_normal(m[p]), fallback=True))
        return out
    st["b"] = draw(st["x"])

    def step():
        x, b = st["x"], st["b"]
        taus = np.stack([O.tau_full(b[p], gw[p]) for p in range(P)])
        if kind == "curn_red":
            rr, _ = (_red_fast if fast else O.rho_grid_cdf_red)(taus, 10 ** (2 * x[rind]), rng.random((P, 30)),
                                                                 1e-20, 1e-8)
            x[hind] = 0.5 * np.log10(rr.ravel())
        irn = (np.stack([10 ** (2 * x[hind[p * 30:(p + 1) * 30]]) for p in range(P)])
               if kind == "curn_red" else np.zeros_like(taus))
        if fast and kind == "curn":               # the same CDF from the tau sums (irn = 0), as the GPU's
            rr, _ = O.rho_grid_cdf_curn_sum(taus.sum(0), P, rng.random(30), 1e-18, 1e-8)   # curn_mode='sum'
        else:
            rr, _ = (_curn_fast if fast else O.rho_grid_cdf_curn)(taus, irn, rng.random(30), 1e-18, 1e-8)
        x[rind] = 0.5 * np.log10(rr)
        st["b"] = draw(x)
    return step, lambda: st["x"][rind], f"45-pulsar {kind} sweeps (oracle restatement of pta_gibbs.py:664-704)"


def pta_mh(aclength=20, fast=False):
    """configs[3] with the reference's default redsample='mh' (pta_gibbs.py:278-340, 664-704):
    per sweep ``aclength`` single-parameter Metropolis steps over every pulsar's power-law
    (log10_A, gamma), each re-evaluating the SUMMED marginalised likelihood of all 45 pulsars
    (get_lnlikelihood :577-621, Cholesky per pulsar, TNT reset and recomputed each sweep), then the
    CURN grid draw with the power-law irn and the SVD b draws.  ``fast`` (ESS runs): TNT once, and a
    step re-evaluates only the moved pulsar's term of the summed likelihood (the others' terms are
    memoised on their phi) -- the same acceptance ratio, so the same Markov kernel."""
    import numpy as np
    from oracle import gibbs_oracle as O
    from pulsar_timing_gibbsspec_amd import synthetic
    from pulsar_timing_gibbsspec_amd.plumbing import uniform_bounds
    p_ = synthetic.array_pta(kind="curn_plred", seed=0)
    T, N, R = p_.get_basis(), p_.get_ndiag({}), p_.get_residuals()
    P = len(T)
    names = p_.param_names
    by_name = {q.name: q for q in p_.params}
    rind = np.array([i for i, n in enumerate(names) if "rho" in n and "gw" in n])
    hind = np.array([i for i, n in enumerate(names) if "red" in n and ("log10_A" in n or "gamma" in n)])
    lo = np.array([uniform_bounds(by_name[names[i]])[0] for i in hind])
    hi = np.array([uniform_bounds(by_name[names[i]])[1] for i in hind])
    red_sigs = [s for s in (p_.signals[k] for k in p_.signals) if "red" in s.name]
    hp = [np.array([i for i in hind if names[i].startswith(p_.pulsars[p] + "_")]) for p in range(P)]
    rng = np.random.default_rng(os.getpid())
    x = rng.uniform(-9, -4, len(names))
    x[hind] = rng.uniform(lo, hi)
    m = [t.shape[1] for t in T]
    gw = [np.arange(mm - 60, mm) for mm in m]
    st = dict(x=x)

    def phis(x):
        return p_.get_phi(p_.map_params(x))

    bd = _bdraw_fast if fast else O.bdraw_svd

    def draw(x, TD):
        return [bd(TD[p][0], TD[p][1], 1.0 / ph, rng.standard_normal(m[p]), fallback=True)
                for p, ph in enumerate(phis(x))]

    def lnprior(x):
        v = x[hind]
        return 0.0 if np.all((v >= lo) & (v <= hi)) else -np.inf
    TD0 = [O.tnt(T[p], N[p], R[p]) for p in range(P)]
    st["b"] = draw(x, TD0)

    def step():
        x, b = st["x"], st["b"]
        TD = TD0 if fast else [O.tnt(T[p], N[p], R[p]) for p in range(P)]   # reset + recompute (:672-673)
        memo = {}

        def term(p, ph):
            return O.lnlike_fullmarg(R[p], N[p], TD[p][0], TD[p][1], 1.0 / ph, float(np.sum(np.log(ph))))

        def lnlike(xx):
            if not fast:
                return sum(term(p, ph) for p, ph in enumerate(phis(xx)))
            tot, params = 0.0, None             # only the moved pulsar's term is new within the block
            for p in range(P):
                key = (p, xx[hp[p]].tobytes())
                if key not in memo:
                    params = params if params is not None else p_.map_params(xx)
                    memo[key] = term(p, np.asarray(p_.models[p].get_phi(params), float))
                tot += memo[key]
            return tot
        steps = [(rng.choice([0.1, 0.5, 1, 3, 10], p=[.1, .15, .5, .15, .1]), rng.choice(hind),
                  rng.standard_normal(), rng.random()) for _ in range(aclength)]
        x = O.white_mh(x, hind, steps, lnlike, lnprior)
        taus = np.stack([O.tau_full(b[p], gw[p]) for p in range(P)])
        irn = np.stack([np.asarray(s.get_phi(p_.map_params(x)), float)[::2] for s in red_sigs])
        rr, _ = (_curn_fast if fast else O.rho_grid_cdf_curn)(taus, irn, rng.random(30), 1e-18, 1e-8)
        x[rind] = 0.5 * np.log10(rr)
        st["x"], st["b"] = x, draw(x, TD)
    return step, lambda: st["x"][rind], (f"45-pulsar CURN + power-law red sweeps with {aclength} red MH steps "
                                         "(oracle restatement of pta_gibbs.py:278-340, 577-621, 664-704)")


def config5(fast=False):
    """configs[4]: one pulsar's sweep (10^4 TOAs, m = 216, 20 white MH steps, each
    recomputing r - T b and the white likelihood as pulsar_gibbs.py:523-546 does); the
    rate is reported per 200-pulsar array sweep (x 1/200)."""
    import numpy as np
    from oracle import gibbs_oracle as O
    from pulsar_timing_gibbsspec_amd import synthetic
    d = synthetic.config5_array(n_psr=1, seed=1)
    T, r, sig, bk = d["T"][0], d["r"][0], d["sigma"][0], d["backend"][0]
    rng = np.random.default_rng(os.getpid())
    st = dict(x=d["x0"][0].copy())
    gw = d["gw_cols"]
    wind = [w[0] for w in d["white"]]
    nb = len(wind) // 2
    lo = np.array([w[3] for w in d["white"]])
    hi = np.array([w[4] for w in d["white"]])
    m = T.shape[1]

    def N_of(xx):
        return O.ndiag_white(sig, bk, xx[[2 * k for k in range(nb)]], xx[[2 * k + 1 for k in range(nb)]])

    def step():
        x = st["x"]
        TNT, dd = O.tnt(T, N_of(x), r)
        ph = np.full(m, 1e-40)
        ph[:gw.size * 2] = 1 / np.repeat(10 ** (2 * x[gw]), 2)
        b = (_bdraw_fast if fast else O.bdraw_svd)(TNT, dd, ph, rng.standard_normal(m), fallback=True)
        ll0 = O.lnlike_white(r, T, b, N_of(x))
        for _ in range(20):
            q = x.copy()
            j = rng.integers(len(wind))
            q[wind[j]] += rng.standard_normal() * 0.05 * len(wind) * rng.choice([0.1, 0.5, 1, 3, 10])
            if lo[j] <= q[wind[j]] <= hi[j]:
                ll1 = O.lnlike_white(r, T, b, N_of(q))
                if ll1 - ll0 > np.log(rng.random()):
                    x, ll0 = q, ll1
        x[gw] = 0.5 * np.log10(O.rho_analytic(O.tau_half(b, np.arange(2 * gw.size)), rng.random(gw.size),
                                              d["rhomin"], d["rhomax"]))
        st["x"] = x
    return step, lambda: st["x"][gw], ("single-pulsar sweeps (10^4 TOAs, m=216, 20 white MH steps; "
                                       "pulsar_gibbs.py:656-698 + :373-404) scaled to the 200-pulsar array")


def _ecorr(white, aclength=10, fast=False):
    """the ECORR sweep (notebook order), optionally with the white MH block."""
    import numpy as np
    from oracle import gibbs_oracle as O
    from pulsar_timing_gibbsspec_amd import synthetic
    p_ = synthetic.ecorr_pulsar_pta("J1713+0747", seed=0, white_vary=white)
    T, r = p_.get_basis()[0], p_.get_residuals()[0]
    names = p_.param_names
    ebk = p_.signals["J1713+0747_basis_ecorr"].epoch_backend
    eind = [i for i, n in enumerate(names) if "ecorr" in n]
    ef_i = [i for i, n in enumerate(names) if n.endswith("efac")]
    eq_i = [i for i, n in enumerate(names) if "equad" in n]
    wind = sorted(ef_i + eq_i)
    gw = np.array([i for i, n in enumerate(names) if "rho" in n])
    m, ne = T.shape[1], ebk.size
    gwid = ne + np.arange(2 * gw.size)
    lo = np.array([0.1 if i in ef_i else -8.5 for i in range(len(names))])
    hi = np.array([5.0 if i in ef_i else -5.0 for i in range(len(names))])
    rng = np.random.default_rng(os.getpid())
    x = np.zeros(len(names))
    x[ef_i], x[eq_i], x[eind] = 1.0, -7.0, -6.3
    x[gw] = rng.uniform(-9, -4, gw.size)
    N_fixed = None if white else p_.get_ndiag()[0]
    wn = p_.models[0].white[0]

    def N_of(xx):
        return O.ndiag_white(wn.sigma, wn.backends, xx[ef_i], xx[eq_i]) if white else N_fixed

    def phi(xx):
        ph = np.full(m, 1e40)
        ph[:ne] = (10.0 ** (2.0 * xx[eind]))[ebk]
        ph[gwid] = np.repeat(10.0 ** (2.0 * xx[gw]), 2)
        return ph

    def prior(ind):
        return lambda xx: 0.0 if np.all((xx[ind] >= lo[ind]) & (xx[ind] <= hi[ind])) else -np.inf

    def steps(ind):
        return [(rng.choice([0.1, 0.5, 1, 3, 10], p=[.1, .15, .5, .15, .1]), rng.choice(ind),
                 rng.standard_normal(), rng.random()) for _ in range(aclength)]
    TNT, dd = O.tnt(T, N_of(x), r)
    TD0 = (TNT, dd) if fast and not white else None      # N fixed without the white block
    bd = _bdraw_fast if fast else O.bdraw_svd
    st = dict(x=x, b=bd(TNT, dd, 1.0 / phi(x), rng.standard_normal(m), fallback=True))

    def step():
        x, b = st["x"], st["b"]
        if white:
            x = O.white_mh(x, wind, steps(wind), lambda xx: O.lnlike_white(r, T, b, N_of(xx)), prior(wind))
        N = N_of(x)
        TNT, dd = TD0 or O.tnt(T, N, r)

        def lnl(xx):
            ph = phi(xx)
            return O.lnlike_fullmarg(r, N, TNT, dd, 1.0 / ph, np.sum(np.log(ph)))
        x = O.white_mh(x, eind, steps(eind), lnl, prior(eind))
        x[gw] = 0.5 * np.log10(O.rho_analytic(O.tau_half(b, gwid), rng.random(gw.size), 1e-18, 1e-8))
        st["x"], st["b"] = x, bd(TNT, dd, 1.0 / phi(x), rng.standard_normal(m), fallback=True)
    what = "white + ECORR" if white else "ECORR"
    return step, lambda: st["x"][gw], (f"single-chain {what} sweeps (m={m}, {ne} epochs, {aclength} MH steps per "
                                       "block, oracle restatement of the notebook sampler)")


KINDS = {
    "single": single,
    "indep": indep,
    "curn": lambda fast=False: pta("curn", fast=fast),
    "curn_red": lambda fast=False: pta("curn_red", fast=fast),
    "curn_plred": lambda fast=False: pta_mh(fast=fast),
    "config5": config5,
    "ecorr": lambda fast=False: _ecorr(False, fast=fast),
    "ecorr_white": lambda fast=False: _ecorr(True, fast=fast),
}
# rates are reported per unit of the BASELINE metric: config5's single-pulsar sweep is 1/200 of an
# array sweep
PER_SWEEP = {"config5": 1.0 / 200.0}


def rate(kind, seconds):
    """(iterations, seconds, what) of one single-thread process running loop ``kind``."""
    step, _, what = KINDS[kind]()
    it, el = _loop(step, seconds)
    return it * PER_SWEEP.get(kind, 1.0), el, what


def ess_rows(kind, burn, sweeps, path):
    """One chain of the port (``fast`` variant: same Markov kernel) for the ESS leg: ``burn`` sweeps
    dropped, then the log10 rho columns of ``sweeps`` sweeps saved to ``path`` (.npy, sweeps x bins)."""
    import numpy as np
    step, get_x, what = KINDS[kind](fast=True)
    for _ in range(burn):
        step()
    rows = np.empty((sweeps, len(get_x())))
    t0 = time.perf_counter()
    for i in range(sweeps):
        step()
        rows[i] = get_x()
    el = time.perf_counter() - t0
    np.save(path, rows)
    return dict(burn_in=burn, sweeps=sweeps, seconds=el, what=what, path=path)


ESS_CHAINS = 6              # independent CPU chains (processes) per line


class EssPool:
    """The CPU ESS leg: ``chains`` single-thread processes per line (each one chain of the port,
    fast variant), at most ``max_procs`` running at once (the box's CPU share minus the GPU driver's
    thread), started in submission order by a background thread while the GPU lines run."""

    def __init__(self, max_procs, workdir):
        import threading
        self.max_procs, self.workdir = max(1, int(max_procs)), workdir
        os.makedirs(workdir, exist_ok=True)
        self.queue, self.procs, self.lock = [], {}, threading.Lock()
        self.t0 = {}
        threading.Thread(target=self._run, daemon=True).start()

    def submit(self, kind, chains=ESS_CHAINS):
        from pulsar_timing_gibbsspec_amd.diagnostics import ESS_RUN
        burn, sweeps = ESS_RUN[kind]
        with self.lock:
            for c in range(chains):
                self.queue.append((kind, c, burn, sweeps))
            self.procs.setdefault(kind, [])

    def _run(self):
        env = dict(os.environ, OPENBLAS_NUM_THREADS="1", OMP_NUM_THREADS="1", MKL_NUM_THREADS="1",
                   PYTHONPATH=ROOT + os.pathsep + os.environ.get("PYTHONPATH", ""))
        while True:
            with self.lock:
                running = sum(p.poll() is None for ps in self.procs.values() for p, _ in ps)
                while self.queue and running < self.max_procs:
                    kind, c, burn, sweeps = self.queue.pop(0)
                    path = os.path.join(self.workdir, f"ess_{kind}_{c}.npy")
                    p = subprocess.Popen([sys.executable, "-m", "oracle.cpu_baseline", kind, "ess", str(burn),
                                          str(sweeps), path], cwd=ROOT, env=env, stdout=subprocess.PIPE,
                                         stderr=subprocess.PIPE, text=True)
                    self.procs[kind].append((p, path))
                    self.t0.setdefault(kind, time.time())
                    running += 1
            time.sleep(0.5)

    def collect(self, kind, timeout=1200):
        """Wait for the line's chains; pooled ESS record (diagnostics.ess_summary) or an error."""
        import numpy as np
        from pulsar_timing_gibbsspec_amd.diagnostics import ess_summary
        deadline = time.time() + timeout
        while True:
            with self.lock:
                pending = any(q[0] == kind for q in self.queue)
                ps = list(self.procs.get(kind, []))
            if not pending and all(p.poll() is not None for p, _ in ps):
                break
            if time.time() > deadline:
                for p, _ in ps:
                    if p.poll() is None:
                        p.kill()
                return {"error": "timed out"}
            time.sleep(0.5)
        rows, info, errs = [], None, []
        for p, path in ps:
            o, e = p.communicate()
            if p.returncode != 0:
                errs.append(e.strip().splitlines()[-1][:300] if e.strip() else f"exit {p.returncode}")
                continue
            info = json.loads(o.strip().splitlines()[-1])
            rows.append(np.load(path))
            os.remove(path)
        if not rows:
            return {"error": errs[0] if errs else "no chains"}
        X = np.stack(rows)                               # (chains, sweeps, bins)
        rec = ess_summary(X, info["burn_in"])
        rec.update(ess_per_sweep=rec["per_chain_sweep_min_bin"], seconds_per_chain=info["seconds"],
                   what=info["what"], wall_s=time.time() - self.t0.get(kind, time.time()),
                   note="independent single-thread processes of the port's fast variant (TNT cached where N "
                        "is fixed; the curn_plred MH step re-evaluates only the moved pulsar's term) -- the "
                        "same Markov kernel as the throughput loop")
        if errs:
            rec["failed_chains"] = len(errs)
        return rec


def host_cores():
    """Cores this process may use: the affinity set, capped by the box's CPU share
    (GS_CPU_CORES, else OMP_NUM_THREADS when it is > 1 -- gpurun sets 16 -- else all)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    cap = os.environ.get("GS_CPU_CORES") or (os.environ.get("OMP_NUM_THREADS")
                                              if int(os.environ.get("OMP_NUM_THREADS", "1")) > 1 else None)
    return max(1, min(n, int(cap))) if cap else n


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def aggregate(kind, seconds, cores=None):
    """Run ``cores`` single-thread processes of loop ``kind`` at once; return the
    cpu_baseline record (value = sum of their rates, iterations/s)."""
    cores = host_cores() if cores is None else int(cores)
    env = dict(os.environ, OPENBLAS_NUM_THREADS="1", OMP_NUM_THREADS="1", MKL_NUM_THREADS="1",
               PYTHONPATH=ROOT + os.pathsep + os.environ.get("PYTHONPATH", ""))
    procs = [subprocess.Popen([sys.executable, "-m", "oracle.cpu_baseline", kind, str(seconds)], cwd=ROOT, env=env,
                              stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True) for _ in range(cores)]
    outs, errs = [], []
    for p in procs:
        o, e = p.communicate(timeout=seconds * 10 + 300)
        if p.returncode != 0:
            errs.append(e[-2000:])
            continue
        outs.append(json.loads(o.strip().splitlines()[-1]))
    if not outs:
        raise RuntimeError(f"cpu baseline {kind} failed: {errs[0]}")
    # a process that died (e.g. a LAPACK error the reference would also have raised) is left
    # out; the aggregate is the survivors' rate scaled to all cores, and says so
    rates = [o["it"] / o["el"] for o in outs]
    extra = {} if not errs else {"failed_processes": len(errs), "error": errs[0].strip().splitlines()[-1][:300]}
    return dict(value=float(sum(rates) * cores / len(outs)), unit="iters/s", cores=cores, kind="port",
                per_process=float(sum(rates) / len(rates)), cpu=cpu_model(), **extra,
                sample=f"{cores} concurrent single-thread processes x {seconds:.0f} s of {outs[0]['what']}; "
                       f"value = sum of their rates (numpy/OpenBLAS, OPENBLAS_NUM_THREADS=1 each)")


def main():
    kind = sys.argv[1]
    if len(sys.argv) > 2 and sys.argv[2] == "ess":
        print(json.dumps(ess_rows(kind, int(sys.argv[3]), int(sys.argv[4]), sys.argv[5])))
        return
    it, el, what = rate(kind, float(sys.argv[2]))
    print(json.dumps(dict(it=it, el=el, what=what)))


if __name__ == "__main__":
    main()
