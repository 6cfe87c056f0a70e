"""PTABlockGibbs' single-call API (update_b, update_rho_params, get_lnlikelihood; pta_gibbs.py:181-214,
512-548, 577-621) on a FRESH sampler, for the models whose phiinv carries per-pulsar red noise
(curn_red: red free spectrum; curn_plred: power-law red noise, the reference's default
redsample='mh').  Each call must see the red phi of the x it is given, not a buffer left from an
earlier call (or never written).

* get_lnlikelihood on a fresh sampler and after calls at other states: 1e-9 relative of the
  oracle's lnlike_fullmarg summed over pulsars (pulsar_gibbs.py:569-610 restated);
* update_b's law at x: with every chain at the same x, the whitened residuals
  w = L^T (b - Sigma^-1 d) (Sigma = L L^T at x's phiinv) of 2048 chains have E|w|^2 = m;
  a stale or garbage red phi moves it by orders of magnitude;
* update_rho_params on a power-law engine runs (it used to pass a NULL red-column table) and
  keeps the common spectrum inside its prior.
Needs an MI355X."""
import numpy as np
import pytest

from oracle import gibbs_oracle as O
from tests.parity_data import refined_mean

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


def _sampler(kind, n_psr=5, C=1, seed=4):
    from pulsar_timing_gibbsspec_amd import PTABlockGibbs, synthetic
    pta = synthetic.array_pta(kind=kind, n_psr=n_psr, seed=2)
    gb = PTABlockGibbs(pta, hypersample="conditional", redsample="conditional" if kind == "curn_red" else "mh",
                       nchains=C, seed=seed)
    return pta, gb


def _x(gb, rng):
    x = np.concatenate([np.atleast_1d(p.sample()).ravel() for p in gb.params])
    # keep the red powers in a range where they matter against the common spectrum
    for i, n in enumerate(gb.param_names):
        if "red_noise_log10_A" in n:
            x[i] = rng.uniform(-15.0, -13.0)
        elif "red_noise_gamma" in n:
            x[i] = rng.uniform(2.0, 5.0)
        elif "red_noise_log10_rho" in n:
            x[i] = rng.uniform(-7.5, -5.0)
    return x


def _oracle_lnl(pta, gb, x):
    prm = gb.map_params(x)
    T, N, r = pta.get_basis(prm), pta.get_ndiag(prm), pta.get_residuals()
    ph = pta.get_phiinv(prm, logdet=True)
    tot = 0.0
    for p in range(len(T)):
        TNT, d = O.tnt(T[p], N[p], r[p])
        tot += O.lnlike_fullmarg(r[p], N[p], TNT, d, ph[p][0], ph[p][1])
    return tot


@pytest.mark.parametrize("kind", ["curn_red", "curn_plred"])
def test_single_call_lnlikelihood_fresh_and_moved(kind):
    pta, gb = _sampler(kind)
    rng = np.random.default_rng(1)
    for _ in range(3):                       # fresh sampler first, then after other states
        x = _x(gb, rng)
        got, want = gb.get_lnlikelihood(x), _oracle_lnl(pta, gb, x)
        assert abs(got - want) <= 1e-9 * abs(want), (kind, got, want)
        gb.update_b(_x(gb, rng))             # leaves the engine at another x


@pytest.mark.parametrize("kind", ["curn_red", "curn_plred"])
def test_single_call_update_b_law(kind):
    C = 2048
    pta, gb = _sampler(kind, n_psr=4, C=C)
    rng = np.random.default_rng(2)
    x = _x(gb, rng)
    gb.update_b(x)                           # fresh sampler: the first call
    eng = gb._api_engine
    prm = gb.map_params(x)
    T, N, r = pta.get_basis(prm), pta.get_ndiag(prm), pta.get_residuals()
    ph = pta.get_phiinv(prm, logdet=False)
    b = eng.b.cpu().numpy().reshape(eng.P, C, -1)
    for p in range(eng.P):
        TNT, d = O.tnt(T[p], N[p], r[p])
        S = TNT + np.diag(ph[p])
        m = S.shape[0]
        mu = refined_mean(S, d)
        L = np.linalg.cholesky(S)
        w = (b[p, :, :m] - mu) @ L           # rows: (L^T (b - mu))^T
        chi2 = np.mean(np.sum(w * w, axis=1))
        assert abs(chi2 - m) < 6.0 * np.sqrt(2.0 * m / C), (kind, p, chi2, m)


def test_update_rho_params_powerlaw():
    pta, gb = _sampler("curn_plred", n_psr=4)
    rng = np.random.default_rng(3)
    x = _x(gb, rng)
    gb._b = gb.update_b(x)
    xn = gb.update_rho_params(x)
    rind = gb.get_rho_param_indices()
    lo, hi = np.log10(gb.rhomin_gw) / 2, np.log10(gb.rhomax_gw) / 2
    assert np.all(np.isfinite(xn))
    assert np.all((xn[rind] >= lo) & (xn[rind] <= hi))
    assert not np.array_equal(xn[rind], x[rind])
    other = np.setdiff1d(np.arange(x.size), rind)
    assert np.array_equal(xn[other], x[other])


def test_update_hyper_params_rejects_nonpositive_iters():
    _, gb = _sampler("curn_plred", n_psr=3)
    x = _x(gb, np.random.default_rng(5))
    with pytest.raises(ValueError):
        gb.update_hyper_params(x, iters=0)
