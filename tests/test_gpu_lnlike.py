""" Marginalised likelihood on the device (gs_lnlike_marg) against the
reference's own values: tests/golden/likelihoods_j1713.npz holds
PulsarBlockGibbs.get_lnlikelihood_fullmarg (pulsar_gibbs.py:569-610) at several
parameter vectors (white noise varied), and the oracle restates it (oracle.lnlike_fullmarg,
pinned to those values in test_oracle_golden.py::test_likelihoods)."""
import numpy as np
import pytest

from oracle import gibbs_oracle as O
from tests.conftest import golden, gpu_available

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    if not gpu_available():
        pytest.skip("no GPU")
    from pulsar_timing_gibbsspec_amd import _lib
    return _lib.Context(0, seed=3)


def _N(g, x):
    names = list(g["param_names"])
    ef = np.array([x[names.index(f"J1713+0747_b{i}_efac")] for i in range(3)])
    eq = np.array([x[names.index(f"J1713+0747_b{i}_log10_tnequad")] for i in range(3)])
    return ef[g["backends"]] ** 2 * g["sigma"] ** 2 + 10 ** (2 * eq[g["backends"]])


def _rho(g, x):
    names = list(g["param_names"])
    return x[[names.index(f"gw_log10_rho_{i}") for i in range(30)]]


def test_lnlike_marg_matches_reference(ctx):
    """Device value == the reference's get_lnlikelihood_fullmarg to 1e-10 relative."""
    import torch
    from pulsar_timing_gibbsspec_amd.engine import DeviceModel
    g = golden("likelihoods_j1713.npz")
    T, r = g["T"], g["r"]
    m = T.shape[1]
    for k in range(g["x"].shape[0]):
        x = g["x"][k]
        model = DeviceModel(ctx, [T], [_N(g, x)], [r], [np.arange(60)], [np.full(m - 60, 1e-40)])
        ph = 1.0 / np.repeat(10 ** (2 * _rho(g, x)), 2)
        lnl, info = model.lnlike_marg(torch.as_tensor(ph[None], device=ctx.device), 1)
        assert int(info[0]) == 0
        assert np.isclose(float(lnl[0]), g["marg"][k], rtol=1e-10, atol=0), (k, float(lnl[0]), g["marg"][k])


def test_lnlike_marg_batch_and_failure(ctx):
    """Many rho vectors at one N in one launch == the oracle; a non-PD system -> -inf."""
    import torch
    from pulsar_timing_gibbsspec_amd.engine import DeviceModel
    g = golden("likelihoods_j1713.npz")
    T, r = g["T"], g["r"]
    m = T.shape[1]
    N = _N(g, g["x"][0])
    model = DeviceModel(ctx, [T], [N], [r], [np.arange(60)], [np.full(m - 60, 1e-40)])
    TNT, d = O.tnt(T, N, r)
    rng = np.random.default_rng(5)
    C = 37
    rho = rng.uniform(-9, -4, (C, 30))
    ph = 1.0 / np.repeat(10 ** (2 * rho), 2, axis=1)
    ph[7, 11] = -1e30                      # system 7: Sigma not positive definite
    lnl, info = model.lnlike_marg(torch.as_tensor(ph, device=ctx.device), C)
    lnl, info = lnl.cpu().numpy(), info.cpu().numpy()
    for c in range(C):
        phiinv = np.concatenate([ph[c], np.full(m - 60, 1e-40)])
        if c == 7:
            assert info[c] > 0 and lnl[c] == -np.inf
            continue
        want = O.lnlike_fullmarg(r, N, TNT, d, phiinv, float(np.sum(np.log(1.0 / phiinv))))
        assert info[c] == 0
        assert np.isclose(lnl[c], want, rtol=1e-10, atol=0), (c, lnl[c], want)
