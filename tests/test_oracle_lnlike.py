"""CPU: the oracle's batched phi-dependent likelihood (lnlike_phi_batch, the grid posterior behind
tests/test_gpu_pta_mh_law.py) against its plain restatement lnlike_fullmarg (pulsar_gibbs.py:569-610,
the per-pulsar term of pta_gibbs.py:577-621): differences between phi rows agree, so the dropped part
is a constant."""
import numpy as np

from oracle import gibbs_oracle as O


def test_lnlike_phi_batch_equals_fullmarg_up_to_a_constant():
    from pulsar_timing_gibbsspec_amd import synthetic
    pta = synthetic.array_pta(kind="curn_plred", n_psr=2, seed=0)
    T, N, R = pta.get_basis({}), pta.get_ndiag({}), pta.get_residuals()
    sig = [s for s in (pta.signals[k] for k in pta.signals) if "red" in s.name][1]
    TNT, d = O.tnt(T[1], N[1], R[1])
    m = TNT.shape[0]
    gwid = np.arange(m - 60, m)
    pf = O.prefix_factor(TNT, d, gwid, np.full(m - 60, 1e-40))
    rng = np.random.default_rng(0)
    rows, full = [], []
    for _ in range(7):
        gw = 10.0 ** rng.uniform(-16, -13, 30)
        red = synthetic.powerlaw_phi(sig.freqs, sig.Tspan, rng.uniform(-16, -13), rng.uniform(1, 6))
        phi = np.repeat(gw + red, 2)
        rows.append(phi)
        phiinv = np.concatenate([np.full(m - 60, 1e-40), 1.0 / phi])
        logdet = np.sum(np.log(phi)) + (m - 60) * np.log(1e40)
        full.append(O.lnlike_fullmarg(R[1], N[1], TNT, d, phiinv, logdet))
    got = O.lnlike_phi_batch(pf, np.array(rows), chunk=3)
    full = np.array(full)
    assert np.allclose(got - got[0], full - full[0], rtol=0, atol=1e-6 * np.abs(full).max() * 1e-3)
