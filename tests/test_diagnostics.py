"""The bench's ESS estimator (diagnostics.pooled_iat / ess_table): pooled ACF over independent
chains, Sokal window, Sokal's standard error -- checked on AR(1) chains, whose IAT is known in
closed form: tau = (1 + a) / (1 - a)."""
import numpy as np

from pulsar_timing_gibbsspec_amd.diagnostics import ess_compare, ess_summary, ess_table, pooled_iat


def _ar1(rng, a, chains, n):
    x = np.empty((chains, n))
    x[:, 0] = rng.standard_normal(chains) / np.sqrt(1 - a * a)
    e = rng.standard_normal((chains, n))
    for t in range(1, n):
        x[:, t] = a * x[:, t - 1] + e[:, t]
    return x


def test_pooled_iat_recovers_ar1():
    rng = np.random.default_rng(0)
    for a in (0.5, 0.9, 0.97):
        tau_true = (1 + a) / (1 - a)
        C, n = 64, int(200 * tau_true)
        tau, M = pooled_iat(_ar1(rng, a, C, n))
        se = tau * np.sqrt(2 * (2 * M + 1) / (C * n))
        assert abs(tau - tau_true) < 3 * se + 0.01 * tau_true, (a, tau, tau_true, se)
        assert M >= 5 * tau * 0.99


def test_standard_error_covers_the_spread():
    """Over independent replicas the ESS estimates scatter by no more than about the standard error
    the estimator reports (the larger of Sokal's and the spread over chain groups: within a factor
    1.6 below, 2.5 above), and sit within 3 SE of 1/tau."""
    rng = np.random.default_rng(1)
    a = 0.9
    f_true = (1 - a) / (1 + a)
    est, ses = [], []
    for _ in range(24):
        X = _ar1(rng, a, 4, 1200)[:, :, None]       # like the CPU leg: few chains, ~60 tau each
        e, se = ess_table(X)
        est.append(e[0])
        ses.append(se[0])
    est, ses = np.array(est), np.array(ses)
    assert 1 / 2.5 < np.std(est) / np.mean(ses) < 1.6
    assert abs(np.mean(est) - f_true) < 3 * np.mean(ses) / np.sqrt(len(est)) + 0.02 * f_true


def test_summary_and_compare():
    rng = np.random.default_rng(2)
    X = np.stack([_ar1(rng, a, 8, 3000) for a in (0.5, 0.9, 0.7)], axis=2)
    Y = np.stack([_ar1(rng, a, 4, 3000) for a in (0.5, 0.9, 0.7)], axis=2)
    g, c = ess_summary(X, 0), ess_summary(Y, 0)
    assert g["bin"] == 1 and c["bin"] == 1
    cmp_ = ess_compare(g, c)
    assert abs(cmp_["z"]) < 3 and cmp_["bin"] == 1
    assert ess_compare(g, ess_summary(Y[:, :, :2], 0)) is None
