"""Chain diagnostics (host-side metric; the reference used the absent ``acor``,
pulsar_gibbs.py:370 and singlepulsar…ipynb:257).

``iat``: integrated autocorrelation time with Sokal's adaptive window
(smallest M with M >= c * tau(M), c = 5); ESS = n / iat.
"""
import numpy as np


def iat(x, c=5.0):
    x = np.asarray(x, float) - np.mean(x)
    n = x.size
    if n < 4:
        return 1.0
    f = np.fft.rfft(x, 2 * n)
    acf = np.fft.irfft(f * np.conj(f))[:n]
    if acf[0] <= 0:
        return 1.0
    acf /= acf[0]
    tau = 2.0 * np.cumsum(acf) - 1.0
    M = np.arange(n)
    ok = M >= c * tau
    if ok.any():
        return float(tau[np.argmax(ok)])
    return float(tau[-1])


# bench.py's ESS runs: (burn-in, recorded sweeps) per chain for each line, the same on the GPU leg and
# the CPU port's (oracle/cpu_baseline.py); recorded >= 50 x the slowest bin's IAT
# (round-6 measurement, profiles/r06a: slowest-bin IAT 29 / 65 / 72 / 261 / 159 / 41 / 42 / 57 sweeps in the
# order below)
ESS_RUN = {"single": (1000, 6000), "indep": (500, 3500), "curn": (500, 5000), "curn_red": (500, 13000),
           "curn_plred": (1000, 8000), "ecorr": (500, 3000), "ecorr_white": (500, 3000), "config5": (500, 3000)}


def pooled_iat(x, c=5.0):
    """(tau, M) of independent chains of one quantity, x: (chains, n).  Each chain's mean is
    removed, the chains' autocovariances (biased, / n) are averaged lag by lag, and tau is read
    off the pooled autocorrelation with Sokal's adaptive window (smallest M with M >= c tau(M)).
    One estimator for every leg of the bench (GPU chains and the CPU port's processes alike)."""
    x = np.atleast_2d(np.asarray(x, float))
    x = x - x.mean(axis=1, keepdims=True)
    C, n = x.shape
    if n < 4:
        return 1.0, 0
    f = np.fft.rfft(x, 2 * n, axis=1)
    acov = np.fft.irfft(f.real ** 2 + f.imag ** 2, axis=1)[:, :n].mean(axis=0)
    if acov[0] <= 0:
        return 1.0, 0
    tau = 2.0 * np.cumsum(acov / acov[0]) - 1.0
    ok = np.arange(n) >= c * tau
    M = int(np.argmax(ok)) if ok.any() else n - 1
    return float(max(tau[M], 1.0)), M


def ess_table(X, c=5.0, groups=16):
    """Per column of X (chains, n, k): the ESS per chain-sweep 1/tau of the pooled chains and its
    standard error -- the larger of (a) Sokal's asymptotic one, var(tau) = 2 (2M + 1) tau^2 / N with
    N = chains x n pooled samples (se(1/tau) = (1/tau) sqrt(2 (2M + 1) / N)), and (b) the spread over
    G = min(chains, groups) disjoint groups of chains, each group's pooled 1/tau (se = std / sqrt(G)),
    which also covers chains that visit a slowly mixing tail only now and then (for which (a), an
    asymptotic formula, reads low with few chains)."""
    X = np.asarray(X)
    C, n, k = X.shape
    out = np.empty(k)
    se = np.empty(k)
    G = min(C, groups)
    parts = np.array_split(np.arange(C), G) if G >= 3 else None
    for j in range(k):
        tau, M = pooled_iat(X[:, :, j], c)
        out[j] = 1.0 / tau
        se[j] = out[j] * np.sqrt(2.0 * (2 * M + 1) / (C * n))
        if parts is not None:
            f = np.array([1.0 / pooled_iat(X[g, :, j], c)[0] for g in parts])
            se[j] = max(se[j], float(np.std(f, ddof=1)) / np.sqrt(G))
    return out, se


def ess_summary(X, burn_in, c=5.0):
    """The bench's ESS record of X (chains, n, k) recorded after ``burn_in`` dropped sweeps: the
    worst column's ESS per chain-sweep with its standard error, and every column's."""
    e, se = ess_table(X, c)
    j = int(np.argmin(e))
    return {"per_chain_sweep_min_bin": float(e[j]), "se": float(se[j]), "bin": j, "chains": int(X.shape[0]),
            "sweeps": int(X.shape[1]), "burn_in": int(burn_in), "per_bin": [float(v) for v in e],
            "se_bin": [float(v) for v in se], "estimator": "pooled ACF over chains, Sokal window c=5"}


def ess_compare(gpu, cpu):
    """z-score of the GPU and CPU ESS per sweep at the GPU's worst column (both from ess_summary),
    and the share of columns that agree within 2 standard errors."""
    g, gs = np.array(gpu["per_bin"]), np.array(gpu["se_bin"])
    h, hs = np.array(cpu["per_bin"]), np.array(cpu["se_bin"])
    if g.shape != h.shape:
        return None
    z = (g - h) / np.sqrt(gs ** 2 + hs ** 2)
    j = int(gpu["bin"])
    return {"bin": j, "gpu": float(g[j]), "gpu_se": float(gs[j]), "cpu": float(h[j]), "cpu_se": float(hs[j]),
            "z": float(z[j]), "frac_bins_within_2se": float(np.mean(np.abs(z) < 2.0))}


def ess(chain, c=5.0):
    """Effective sample size of each column of a (n, k) chain."""
    chain = np.atleast_2d(np.asarray(chain, float))
    if chain.shape[0] == 1:
        chain = chain.T
    return np.array([chain.shape[0] / max(iat(chain[:, k], c), 1.0) for k in range(chain.shape[1])])


def acor(x, maxlag=10):
    """(tau, mean, sigma) of a 1-d chain: restatement of J. Goodman's ``acor``
    algorithm (PyPI ``acor`` 1.1.x, the module pulsar_gibbs.py:370-371 calls; absent
    here and unpinned by the reference): autocovariances C[0..maxlag] over the
    first L - maxlag points, D = C0 + 2 sum C[s], tau = D / C0; while
    tau * 5 >= maxlag the chain is pair-summed (length halves) and the estimate
    recomputed from the coarse chain (D = sigma^2 L / 4 with sigma from the
    recursion).  Chains shorter than 5 * maxlag return the estimate so far."""
    x = np.asarray(x, float).copy()
    return _acor(x, int(maxlag))


def _acor(x, maxlag):
    L = x.size
    mean = float(np.mean(x)) if L else 0.0
    x = x - mean
    if L < 5 * maxlag:
        return 1.0, mean, 0.0
    i_max = L - maxlag
    C = np.array([np.dot(x[:i_max], x[s:s + i_max]) for s in range(maxlag + 1)]) / i_max
    D = C[0] + 2.0 * np.sum(C[1:])
    if C[0] <= 0 or D < 0:
        return 1.0, mean, 0.0
    sigma = np.sqrt(D / L)
    tau = D / C[0]
    if tau * 5 < maxlag:
        return float(tau), mean, float(sigma)
    Lh = L // 2
    xx = x[0:2 * Lh:2] + x[1:2 * Lh:2]
    if Lh < 5 * maxlag:
        return float(tau), mean, float(sigma)
    _, _, sigma = _acor(xx, maxlag)
    D = 0.25 * sigma * sigma * L
    return float(D / C[0]), mean, float(np.sqrt(D / L))


def white_aclength(short_chain, burn=100):
    """aclength_white = max_j int(acor(short_chain[burn:, j])[0])  (pulsar_gibbs.py:370-371)."""
    sc = np.asarray(short_chain, float)[burn:]
    return int(np.max([int(acor(sc[:, j])[0]) for j in range(sc.shape[1])]))
