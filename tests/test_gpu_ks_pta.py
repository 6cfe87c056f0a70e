"""north_star's distributional check on its own target configuration (BASELINE configs[3]):
with independent RNG streams, the marginal posteriors of log10 rho from the device agree with
the reference's under a two-sample KS test per frequency bin.

Reference: a 20k-sweep PTABlockGibbs.sample chain of the reference itself on the 45-pulsar
array (pta_gibbs.py:631-713; tests/golden/make_golden.py --only-pta-long-<kind>, seeded,
single-threaded BLAS), thinned per bin by its own integrated autocorrelation time so its draws
are ~independent.  Device: chains in the bench's modes -- CURN from the tau sums
(curn_mode='sum', the fixed-point sufficient statistic and k_rho_curn_sum_wave), CURN + red
with the default fast grid kernels (k_rho_red_wave, k_rho_curn_fast) -- one draw per
independent chain after burn-in.  Bonferroni over the tested bins.
"""
import numpy as np
import pytest

from tests.conftest import golden

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

ALPHA = 1e-3


def _ref_draws(kind, burn=1000):
    from pulsar_timing_gibbsspec_amd.diagnostics import iat
    g = golden(f"pta_long_{kind}.npz")
    c = g["chain"].astype(np.float64)[burn:]
    out = []
    for k in range(c.shape[1]):
        t = max(1, int(np.ceil(iat(c[:, k]))))
        out.append(c[::t, k])
    return out, list(g["names"]), np.asarray(g["cols"])


def _device_draws(kind, C=2048, sweeps=1500, seed=77):
    from pulsar_timing_gibbsspec_amd import PTABlockGibbs, synthetic
    pta = synthetic.array_pta(kind=kind, seed=0)
    gb = PTABlockGibbs(pta, hypersample="conditional", redsample="conditional" if kind == "curn_red" else "mh",
                       nchains=C, seed=seed)
    rng = np.random.default_rng(seed)
    lo, hi = np.log10(gb.rhomin_gw) / 2, np.log10(gb.rhomax_gw) / 2
    eng = gb._new_engine(np.full(len(gb.param_names), (lo + hi) / 2))
    assert eng.curn_mode == ("sum" if kind == "curn" else "exact")
    # independent starting points over the prior, one per chain
    x = rng.uniform(lo, hi, (C, len(gb.param_names)))
    eng.x.copy_(torch.as_tensor(x, device=eng.ctx.device))
    for _ in range(sweeps):
        eng.sweep()
    assert int(eng.info.abs().sum()) == 0
    return eng.x.cpu().numpy(), list(gb.param_names)


@pytest.mark.parametrize("kind", ["curn", "curn_red"])
def test_pta_posterior_ks_against_reference(kind):
    try:
        ref, names_ref, cols = _ref_draws(kind)
    except FileNotFoundError:
        pytest.skip(f"tests/golden/pta_long_{kind}.npz not generated")
    x, names = _device_draws(kind)
    assert [names[c] for c in cols] == names_ref
    pv = []
    from scipy.stats import ks_2samp
    for j, c in enumerate(cols):
        pv.append(ks_2samp(x[:, c], ref[j]).pvalue)
    pv = np.array(pv)
    assert pv.min() > ALPHA / len(pv), (kind, pv.min(), int(np.argmin(pv)), [len(r) for r in ref][:5])
