"""north_star's distributional check on its own target configuration (BASELINE configs[3]):
with independent RNG streams, the marginal posteriors of log10 rho from the device agree with
the reference's under a two-sample KS test per frequency bin.

Reference: a 20k-sweep PTABlockGibbs.sample chain of the reference itself on the 45-pulsar
array (pta_gibbs.py:631-713; tests/golden/make_golden.py --only-pta-long-<kind>, seeded,
single-threaded BLAS), thinned per bin by its own integrated autocorrelation time so its draws
are ~independent.  Device: chains in the bench's modes -- CURN from the tau sums
(curn_mode='sum', the fixed-point sufficient statistic and k_rho_curn_sum_cert16), CURN + red
with the default certified grid kernels (k_rho_red_cert16, k_rho_curn_fast) -- one draw per
independent chain after burn-in.  Bonferroni over the tested bins.

curn_plred: the reference's DEFAULT model (redsample='mh': per-pulsar power-law red noise by the
Metropolis block, pta_gibbs.py:278-340) on 6 pulsars, against six independent 40k-sweep runs of
the reference's own methods in sample()'s order (make_golden.py --only-pta-long-plred; sample()
itself cannot pass sweep 0 on this path, so the 100 warm-up steps run through the steady-state
branch, aclength_hyper = 20 after), every common log10 rho bin and every pulsar's (log10_A,
gamma); curn_plred45: the same on north_star's 45-pulsar array (configs[3]) against five
independent 20k-sweep reference runs (make_golden.py --only-pta-long-plred --npsr=45), every
common bin and all 90 (log10_A, gamma).  Device: k_hyper_mh with device Philox (no injected draws), the lnL seed from the gated
k_bdraw_tiled draw, k_rho_curn_fast with the power-law irn.
"""
import numpy as np
import pytest

from tests.conftest import golden

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

ALPHA = 1e-3


PLRED_PSR = 6       # the curn_plred reference runs' array (make_golden.pta_long_plred)
# reference runs per curn_plred array size: file pattern, burn-in (sweeps) of the reference rows
# and of the device chains (the power-law red block moves each of 2 x n_psr parameters ~20 / (2 n_psr)
# times per sweep, so the 45-pulsar array burns in over more sweeps)
PLRED = {6: ("pta_long_curn_plred_s*.npz", 1000, 1500), 45: ("pta_long_curn_plred_p45_s*.npz", 4000, 5000)}


def _thin(c, burn):
    from pulsar_timing_gibbsspec_amd.diagnostics import iat
    c = c[burn:]
    return [c[::max(1, int(np.ceil(iat(c[:, k])))), k] for k in range(c.shape[1])]


def _plred_files(n_psr):
    import glob
    import os

    from tests.conftest import GOLDEN
    return sorted(glob.glob(os.path.join(GOLDEN, PLRED[n_psr][0])))


def _ref_draws(kind, burn=1000, n_psr=PLRED_PSR):
    if kind == "curn_plred":
        files = _plred_files(n_psr)
        burn = PLRED[n_psr][1]
        if not files:
            raise FileNotFoundError(PLRED[n_psr][0])
        parts, g = [], None
        for f in files:                         # each independent run thinned by its own IATs
            g = np.load(f, allow_pickle=False)
            parts.append(_thin(g["chain"].astype(np.float64), burn // int(g["thin"])))
        out = [np.concatenate([p[k] for p in parts]) for k in range(len(parts[0]))]
        return out, list(g["names"]), np.asarray(g["cols"])
    g = golden(f"pta_long_{kind}.npz")
    return _thin(g["chain"].astype(np.float64), burn), list(g["names"]), np.asarray(g["cols"])


def _device_draws(kind, C=2048, sweeps=1500, seed=77, n_psr=PLRED_PSR):
    from pulsar_timing_gibbsspec_amd import PTABlockGibbs, synthetic
    if kind == "curn_plred":
        sweeps = PLRED[n_psr][2]
    pta = synthetic.array_pta(kind=kind, seed=0, n_psr=n_psr if kind == "curn_plred" else None)
    gb = PTABlockGibbs(pta, hypersample="conditional", redsample="conditional" if kind == "curn_red" else "mh",
                       nchains=C, seed=seed)
    rng = np.random.default_rng(seed)
    lo, hi = np.log10(gb.rhomin_gw) / 2, np.log10(gb.rhomax_gw) / 2
    eng = gb._new_engine(np.full(len(gb.param_names), (lo + hi) / 2))
    assert eng.curn_mode == ("sum" if kind == "curn" else "exact")
    # independent starting points over the prior, one per chain
    x = rng.uniform(lo, hi, (C, len(gb.param_names)))
    if eng.hyper is not None:
        hs = eng.hyper_spec
        x[:, hs.hind] = rng.uniform(hs.hlo_host, hs.hhi_host, (C, hs.n_h))
        eng.hyper_acl = 20                      # the reference runs' aclength_hyper
    eng.x.copy_(torch.as_tensor(x, device=eng.ctx.device))
    for _ in range(sweeps):
        eng.sweep()
    assert int(eng.info.abs().sum()) == 0
    return eng.x.cpu().numpy(), list(gb.param_names)


@pytest.mark.parametrize("kind,n_psr", [("curn", 45), ("curn_red", 45), ("curn_plred", 6), ("curn_plred", 45)])
def test_pta_posterior_ks_against_reference(kind, n_psr):
    try:
        ref, names_ref, cols = _ref_draws(kind, n_psr=n_psr)
    except FileNotFoundError:
        pytest.skip(f"tests/golden/pta_long_{kind}.npz not generated")
    if kind == "curn_plred" and n_psr == 45:
        assert len(cols) == 30 + 90 and min(len(r) for r in ref) >= 200
    x, names = _device_draws(kind, n_psr=n_psr)
    assert [names[c] for c in cols] == names_ref
    pv = []
    from scipy.stats import ks_2samp
    for j, c in enumerate(cols):
        pv.append(ks_2samp(x[:, c], ref[j]).pvalue)
    pv = np.array(pv)
    assert pv.min() > ALPHA / len(pv), (kind, pv.min(), int(np.argmin(pv)), [len(r) for r in ref][:5])


def _lag1(rows):
    """Pooled lag-1 autocorrelation per column of (chains, n, k) rows, each chain demeaned."""
    x = rows - rows.mean(axis=1, keepdims=True)
    return np.sum(x[:, 1:] * x[:, :-1], axis=(0, 1)) / np.sum(x * x, axis=(0, 1))


@pytest.mark.parametrize("n_psr", [6, 45])
def test_plred_mixing_matches_reference(n_psr):
    """The device's Markov kernel mixes like the reference's on the reference-default model
    (curn_plred, redsample='mh', aclength_hyper 20): the lag-10-sweep autocorrelation of every
    common log10 rho bin and every (log10_A, gamma) agrees with the reference runs (six 40k-sweep
    ones at 6 pulsars, five 20k-sweep ones at 45; their rows are every 10th sweep) within 5 standard
    errors (the reference's from the spread over its runs, floored at 0.01).  ESS per sweep follows
    from these autocorrelations; this is the like-for-like check behind the bench's GPU vs CPU ESS
    figures."""
    from pulsar_timing_gibbsspec_amd import PTABlockGibbs, synthetic
    files = _plred_files(n_psr)
    if len(files) < 3:
        pytest.skip("reference plred runs not generated")
    refs = [np.load(f, allow_pickle=False) for f in files]
    thin, names_ref, cols = int(refs[0]["thin"]), list(refs[0]["names"]), np.asarray(refs[0]["cols"])
    burn = PLRED[n_psr][1] // thin
    r_ref = np.stack([_lag1(g["chain"].astype(np.float64)[burn:][None]) for g in refs])   # (runs, k)
    se = np.maximum(r_ref.std(axis=0, ddof=1) / np.sqrt(len(refs)), 0.01)
    C, rows = 512, 1500
    pta = synthetic.array_pta(kind="curn_plred", seed=0, n_psr=n_psr)
    gb = PTABlockGibbs(pta, nchains=C, seed=19)
    eng = gb._new_engine(np.zeros(len(gb.param_names)))
    assert [gb.param_names[c] for c in cols] == names_ref
    rng = np.random.default_rng(19)
    lo, hi = np.log10(gb.rhomin_gw) / 2, np.log10(gb.rhomax_gw) / 2
    x = rng.uniform(lo, hi, (C, len(gb.param_names)))
    hs = eng.hyper_spec
    x[:, hs.hind] = rng.uniform(hs.hlo_host, hs.hhi_host, (C, hs.n_h))
    eng.hyper_acl = 20
    eng.x.copy_(torch.as_tensor(x, device=eng.ctx.device))
    for _ in range(max(2000, PLRED[n_psr][2])):              # burn-in (>= the reference rows' above)
        eng.sweep()
    rec = torch.empty(rows, C, len(cols), dtype=torch.float64, device=eng.ctx.device)
    ci = torch.as_tensor(cols, dtype=torch.long, device=eng.ctx.device)
    for i in range(rows):
        for _ in range(thin):
            eng.sweep()
        rec[i] = eng.x.index_select(1, ci)
    r_dev = _lag1(rec.cpu().numpy().transpose(1, 0, 2))
    z = np.abs(r_dev - r_ref.mean(axis=0)) / se
    assert z.max() < 5.0, (names_ref[int(np.argmax(z))], float(z.max()), np.round(r_dev, 3), np.round(r_ref.mean(0), 3))
