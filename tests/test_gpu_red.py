""" Power-law intrinsic red noise on the device.

* gs_red_mh's likelihood (nsteps = 0) == the reference's get_lnlikelihood_red
  (pulsar_gibbs.py:549-566) on its own values (tests/golden/red_lnlike_j1713.npz), 1e-12.
* The Metropolis block == the oracle restatement on the same Philox stream
  (oracle.red_mh_philox): identical accept decisions and states (1e-12) for every chain
  whose steps are all further than 1e-9 from an accept/reject tie; both acceptance
  semantics (anchor = 1, the reference's; anchor = 0, textbook).
* anchor = 0 samples the exact conditional p(log10_A, gamma | b, rho): KS test of 4096
  chains' final states against the posterior integrated on a fine host grid.
* update_gwrho_params with a red signal (grid + Gumbel-max, pulsar_gibbs.py:218-234)
  reproduces the reference's draws given its Gumbel uniforms (gumbel_j1713.npz).
* sample() with red noise: warm-up + device sweeps, chain files and prior bounds.
The proposal law restates PTMCMCSampler (absent, unpinned): parity of the jumps is
against the restatement only."""
import numpy as np
import pytest

from oracle import gibbs_oracle as O
from tests.conftest import golden, gpu_available

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gibbs():
    if not gpu_available():
        pytest.skip("no GPU")
    from pulsar_timing_gibbsspec_amd import synthetic
    from pulsar_timing_gibbsspec_amd.pulsar_gibbs import PulsarBlockGibbs
    pta = synthetic.single_pulsar_pta("J1713+0747", seed=0, powerlaw_red=True)
    return PulsarBlockGibbs(pta, seed=11)


def test_red_lnlike_matches_reference(gibbs):
    g = golden("red_lnlike_j1713.npz")
    assert list(gibbs.param_names) == list(g["param_names"])
    for b, x, want in zip(g["b"], g["x"], g["lnl"]):
        gibbs._b = b.copy()
        got = gibbs.get_lnlikelihood_red(x)
        assert abs(got - want) <= 1e-12 * abs(want), (got, want)


def _engine(gibbs, C, cov, de, anchor, rng):
    import torch
    from pulsar_timing_gibbsspec_amd.rednoise import RedJumps
    g = golden("red_lnlike_j1713.npz")
    x0 = g["x"][0]
    ia, ig, lnphi, bounds = gibbs._red_setup(x0)
    jumps = RedJumps(cov, de, bounds, gibbs.ctx.device)
    eng = gibbs._red_engine(x0, C, jumps=jumps)
    eng.anchor = anchor
    m = len(gibbs._b)
    B = rng.standard_normal((C, m)) * 10 ** rng.uniform(-8, -6.5, (C, m))
    X = np.broadcast_to(x0, (C, x0.size)).copy()
    X[:, gibbs.get_gwrho_param_indices()] = rng.uniform(-9, -4, (C, 30))
    X[:, ia] = rng.uniform(-16, -12, C)
    X[:, ig] = rng.uniform(1, 6, C)
    eng.x.copy_(torch.as_tensor(X))
    eng.b[:, :m] = torch.as_tensor(B)
    return eng, X, B, (ia, ig, lnphi, bounds)


@pytest.mark.parametrize("anchor", [1, 0])
def test_red_mh_matches_oracle(gibbs, anchor):
    rng = np.random.default_rng(21 + anchor)
    cov = np.array([[0.4, -0.3], [-0.3, 0.5]])
    de = np.stack([rng.uniform(-16, -12, 200), rng.uniform(1, 6, 200)], axis=1)
    C = 256
    eng, X, B, (ia, ig, lnphi, _) = _engine(gibbs, C, cov, de, anchor, rng)
    eng.it = 7
    eng._tau()
    tau = eng.tau.cpu().numpy()
    eng.red_block(20)
    xg = eng.x.cpu().numpy()
    lg = eng.lnl.cpu().numpy()
    ag = eng.n_acc.cpu().numpy()
    gw_col = gibbs.get_gwrho_param_indices()
    seed = int(gibbs.ctx.seed)
    key = np.array([seed & 0xffffffff, seed >> 32], np.uint32)
    checked = 0
    for c in range(C):
        xo, lo, ao, marg = O.red_mh_philox(X[c], ia, ig, gw_col, tau[:, c], lnphi, eng.jumps.table_host, de,
                                           20, anchor, key, 7, c)
        if marg.min() < 1e-9:
            continue                                       # an accept/reject near-tie
        checked += 1
        assert ag[c] == ao, c
        assert np.allclose(xg[c], xo, rtol=1e-12, atol=1e-12), c
        assert abs(lg[c] - lo) <= 1e-11 * abs(lo), c
    assert checked >= C - 2
    assert 0 < ag.mean() < 20


def test_red_mh_samples_conditional(gibbs):
    """anchor = 0: 4096 chains x 40 blocks from spread starts; the final (log10_A, gamma)
    marginals match the exact conditional posterior (2-D host grid) under a KS test."""
    import torch
    from scipy import stats
    rng = np.random.default_rng(5)
    C = 4096
    cov = np.array([[0.3, -0.2], [-0.2, 0.4]])
    eng, X, B, (ia, ig, lnphi, bounds) = _engine(gibbs, C, cov, np.zeros((0, 2)), 0, rng)
    # one (b, rho) for every chain: the conditional is then the same for all
    eng.b.copy_(eng.b[:1].expand(C, -1).clone())
    xr = eng.x[:1].clone()
    eng.x.copy_(xr.expand(C, -1))
    eng.x[:, ia] = torch.as_tensor(rng.uniform(*bounds[0], C))
    eng.x[:, ig] = torch.as_tensor(rng.uniform(*bounds[1], C))
    eng._tau()
    for s in range(40):
        eng.it = 100 + s
        eng.red_block(20)
    xs = eng.x.cpu().numpy()
    tau = eng.tau[:, 0].cpu().numpy()
    x0 = xr[0].cpu().numpy()
    gwphi = 10 ** (2 * x0[gibbs.get_gwrho_param_indices()])
    def post(la, ga):
        LA, GA = np.meshgrid(la, ga, indexing="ij")
        lirn = (lnphi[1][None, None] * LA[..., None] + lnphi[0]) + lnphi[2] * GA[..., None]
        lr = np.log(tau) - np.logaddexp(lirn, np.log(gwphi))
        lp = np.sum(lr - np.exp(lr), axis=-1)
        return np.exp(lp - lp.max())
    la = np.linspace(*bounds[0], 901)
    ga = np.linspace(*bounds[1], 701)
    p = post(la, ga)                                       # coarse, then refine on the support
    ia_, ig_ = np.nonzero(p > 1e-14)
    la = np.linspace(max(bounds[0][0], la[ia_.min()] - 0.02), min(bounds[0][1], la[ia_.max()] + 0.02), 1501)
    ga = np.linspace(max(bounds[1][0], ga[ig_.min()] - 0.02), min(bounds[1][1], ga[ig_.max()] + 0.02), 1501)
    p = post(la, ga)
    for axis, vals, grid in ((1, xs[:, ia], la), (0, xs[:, ig], ga)):
        pdf = p.sum(axis=axis)
        cdf = np.cumsum(pdf) / pdf.sum()
        stat, pval = stats.kstest(vals, lambda v: np.interp(v, grid, cdf))
        assert pval > 1e-3, (axis, stat, pval)


def test_gumbel_rho_with_red_matches_reference(gibbs):
    g = golden("gumbel_j1713.npz")
    assert list(gibbs.param_names) == list(g["param_names"])
    for c in range(len(g["b"])):
        gibbs._b = g["b"][c].copy()
        xn = gibbs.update_gwrho_params(g["x"][c].copy(), u=g["gumbel_u"][c])
        assert np.array_equal(xn, g["xnew"][c]), c


def test_sample_with_red_noise(gibbs, tmp_path):
    from pulsar_timing_gibbsspec_amd import synthetic
    from pulsar_timing_gibbsspec_amd.pulsar_gibbs import PulsarBlockGibbs
    pta = synthetic.single_pulsar_pta("J1713+0747", seed=0, powerlaw_red=True)
    gb = PulsarBlockGibbs(pta, seed=3, nchains=64)
    np.random.seed(1)
    x0 = np.concatenate([p.sample().flatten() for p in gb.params])
    out = tmp_path / "red"
    gb.red_warmup_iters = 400
    chain = gb.sample(x0, outdir=str(out), niter=201)
    assert chain.shape == (201, x0.size)
    assert np.array_equal(chain[0], x0)
    assert (out / "chain.npy").exists() and np.load(out / "chain.npy").shape[0] == 201
    ia, ig, _, bounds = gb._red_setup(x0)
    cs = gb.chains
    assert (cs[:, :, ia] >= bounds[0][0]).all() and (cs[:, :, ia] <= bounds[0][1]).all()
    assert (cs[:, :, ig] >= bounds[1][0]).all() and (cs[:, :, ig] <= bounds[1][1]).all()
    rho = cs[:, :, gb.get_gwrho_param_indices()]
    assert np.isfinite(rho).all() and (rho >= -9).all() and (rho <= -4).all()
    acc = gb.red_acceptance
    assert acc is not None and 0.0 < acc.mean() < 1.0
    # the chains move (b redrawn through the gate) and differ across chains
    assert np.std(cs[:, -1, ia]) > 0 and np.std(gb.bchains[:, -1, 0]) > 0
