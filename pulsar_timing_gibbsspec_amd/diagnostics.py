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
