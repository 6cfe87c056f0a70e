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
