"""The reference's DEFAULT PTA red-noise block (PTABlockGibbs(redsample='mh'), pta_gibbs.py:278-340 on
get_lnlikelihood :577-621) in PRODUCTION mode -- device Philox, no injected draws -- against its
target law.

test_gpu_pta_mh.py pins every MH decision of k_hyper_mh bit for bit on the reference's captured
draws; it cannot see the Philox branch (the scale from one uniform for choice(sizes, p=probs), the
parameter from floor(u n_h) for choice(hind), the Box-Muller normal, log of the acceptance uniform,
the 64-step proposal table).  Here the common spectrum is frozen and only the block runs, so its
stationary law is known exactly: with phi_gw fixed, the summed likelihood separates over pulsars, so
pulsar p's (log10_A, gamma) has the posterior exp(lnL_p(log10_A, gamma)) on its uniform prior box,
which the oracle evaluates on a 2-D grid (oracle.lnlike_phi_batch: pulsar p's term of
get_lnlikelihood restated from TNT, d and the power-law phi of the facade's own get_phi formula).

4096 independent chains from starts spread over the prior box, 6000 steps each (750 per
parameter) in blocks of 200 (each block re-seeds lnL_p from the current x, as every sweep does);
the final state of each chain is one draw.  KS of each pulsar's log10_A and gamma marginals against
the grid CDFs, Bonferroni over the 2 P marginals.  Needs an MI355X."""
import numpy as np
import pytest

from oracle import gibbs_oracle as O

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

ALPHA = 1e-3


def _grid_marginals(pf, phi_gw, freqs, Tspan, lo, hi, n_coarse=(73, 57), n_fine=(241, 201)):
    """Marginal CDFs of (log10_A, gamma) of exp(lnL(phi_gw + phi_red(log10_A, gamma))) on the prior box:
    a coarse grid locates the mass, a fine grid over the box holding all but ~1e-9 of it integrates."""
    from pulsar_timing_gibbsspec_amd.synthetic import powerlaw_phi

    def lnl_grid(a, g):
        A, G = np.meshgrid(a, g, indexing="ij")
        red = powerlaw_phi(freqs[None, :], Tspan, A.reshape(-1, 1), G.reshape(-1, 1))
        phi = np.repeat(phi_gw[None, :] + red, 2, axis=1)          # (sin, cos) per frequency
        return O.lnlike_phi_batch(pf, phi).reshape(A.shape)

    a = np.linspace(lo[0], hi[0], n_coarse[0])
    g = np.linspace(lo[1], hi[1], n_coarse[1])
    L = lnl_grid(a, g)
    keep = L > L.max() - 25.0
    ia, ig = np.nonzero(keep)
    da, dg = a[1] - a[0], g[1] - g[0]
    a0, a1 = max(lo[0], a[ia.min()] - da), min(hi[0], a[ia.max()] + da)
    g0, g1 = max(lo[1], g[ig.min()] - dg), min(hi[1], g[ig.max()] + dg)
    a = np.linspace(a0, a1, n_fine[0])
    g = np.linspace(g0, g1, n_fine[1])
    L = lnl_grid(a, g)
    w = np.exp(L - L.max())
    pa = np.trapezoid(w, g, axis=1)
    pg = np.trapezoid(w, a, axis=0)

    def cdf(x, p):
        c = np.concatenate([[0.0], np.cumsum(0.5 * (p[1:] + p[:-1]) * np.diff(x))])
        return x, c / c[-1]
    return cdf(a, pa), cdf(g, pg)


def test_hyper_mh_philox_matches_grid_posterior():
    from scipy.stats import kstest

    from pulsar_timing_gibbsspec_amd import PTABlockGibbs, synthetic
    P, C, blocks, nsteps = 4, 4096, 30, 200
    pta = synthetic.array_pta(kind="curn_plred", n_psr=P, seed=0)
    gb = PTABlockGibbs(pta, nchains=C, seed=123)
    names = gb.param_names
    rind = gb.get_rho_param_indices()
    rng = np.random.default_rng(9)
    x0 = np.concatenate([np.atleast_1d(p.sample()).ravel() for p in gb.params])
    # the common spectrum frozen at the simulated GWB's power law (A = 2e-15, gamma = 13/3)
    gw_sig = gb.gw_sig
    x0[rind] = 0.5 * np.log10(synthetic.powerlaw_phi(gw_sig.freqs, gw_sig.Tspan, np.log10(2e-15), 13 / 3))
    eng = gb._new_engine(x0)
    hs = eng.hyper_spec
    x = np.repeat(x0[None], C, axis=0)
    x[:, hs.hind] = rng.uniform(hs.hlo_host, hs.hhi_host, (C, hs.n_h))       # spread starts
    eng.x.copy_(torch.as_tensor(x, device=eng.ctx.device))
    for _ in range(blocks):
        eng.hyper_block(nsteps)
        eng.it += 1                                  # the next block's Philox counters
    xe = eng.x.cpu().numpy()
    assert np.array_equal(xe[:, rind], x[:, rind])   # the block moves only red parameters
    assert np.all(np.isfinite(xe))
    acc = float(eng.hyper.acc_total.sum()) / (C * blocks * nsteps)
    assert 0.05 < acc < 0.95, acc

    params = gb.map_params(x0)
    T, N, R = pta.get_basis(params), pta.get_ndiag(params), pta.get_residuals()
    phi_gw = 10.0 ** (2.0 * x0[rind])
    pv, where = [], []
    for p in range(P):
        sig = gb.red_sig[p]
        TNT, d = O.tnt(T[p], N[p], R[p])
        m = TNT.shape[0]
        gwid = np.asarray(gb.gwid[p])
        pf = O.prefix_factor(TNT, d, gwid, np.full(m - gwid.size, 1e-40))
        j = np.nonzero(hs.hpsr_host == p)[0]
        cols = hs.hind[j]
        ia = j[["log10_A" in names[c] for c in cols].index(True)]
        ig = j[["gamma" in names[c] for c in cols].index(True)]
        lo = (hs.hlo_host[ia], hs.hlo_host[ig])
        hi = (hs.hhi_host[ia], hs.hhi_host[ig])
        (ga, ca), (gg, cg) = _grid_marginals(pf, phi_gw, sig.freqs, sig.Tspan, lo, hi)
        for col, (gx, cx) in ((hs.hind[ia], (ga, ca)), (hs.hind[ig], (gg, cg))):
            pv.append(kstest(xe[:, col], lambda v, gx=gx, cx=cx: np.interp(v, gx, cx)).pvalue)
            where.append(names[col])
    pv = np.array(pv)
    assert pv.min() > ALPHA / len(pv), (pv.min(), where[int(np.argmin(pv))], np.round(pv, 4))
