"""Config 5 path on the GPU (BASELINE configs[4]): NF = 200 free-spectrum blocks
(workspace-tile b-draw, csrc/gibbs_big.hip), the one-pass batched SYRK for per-chain
TNT/d (csrc/gibbs_white.hip), and the independent-pulsar white-noise engine
(white.WhiteArrayChains).

Oracles: the b-draw against the exact (long double) Cholesky draw with the same normals
(tests/parity_data.exact_chol_draw, the draw law of pulsar_gibbs.py:489-520 with the
rotated normals of the golden fixtures); TNT/d against numpy's T.T @ (T / N)
(pulsar_gibbs.py:500-502); the array engine against the single-pulsar engine, which is
itself pinned to the reference's captured run (test_gpu_white.py).  Sizes are cut so
the long-double oracle finishes in seconds; the full 200 x 10^4 x 216 case runs in
bench.py."""
import numpy as np
import pytest

from oracle import gibbs_oracle as O
from tests.conftest import gpu_available
from tests.parity_data import exact_chol_draw, normwise_rel

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    if not gpu_available():
        pytest.skip("no GPU")
    from pulsar_timing_gibbsspec_amd import _lib
    return _lib.Context(0, seed=11)


def _white_N(d, p, x):
    nb = len(d["white"]) // 2
    ef = x[[2 * k for k in range(nb)]]
    eq = x[[2 * k + 1 for k in range(nb)]]
    return O.ndiag_white(d["sigma"][p], d["backend"][p], ef, eq)


@pytest.mark.parametrize("n_f", [40, 100, 104])
def test_big_bdraw_matches_exact_draw(ctx, n_f):
    """gs_bdraw (NF = 80, 200, 208 -> augmented column in the last tile / its own tile)
    == the exact Cholesky draw with the same normals, 1e-9 normwise."""
    import torch
    from pulsar_timing_gibbsspec_amd import synthetic
    from pulsar_timing_gibbsspec_amd.engine import DeviceModel
    d = synthetic.config5_array(n_psr=1, n_toa=900, n_f=n_f, seed=3)
    T, r = d["T"][0], d["r"][0]
    N = d["sigma"][0] ** 2
    NF = 2 * n_f
    m = T.shape[1]
    model = DeviceModel(ctx, [T], [N], [r], [d["fidx"]], [d["phiinv_fixed"]])
    rng = np.random.default_rng(4)
    C = 3
    logrho = rng.uniform(-8.5, -5.0, (C, n_f))
    ph = 1.0 / np.repeat(10 ** (2 * logrho), 2, axis=1)
    z = np.zeros((C, model.ldb))
    z[:, :m] = rng.standard_normal((C, m))
    dev = lambda a: torch.as_tensor(np.ascontiguousarray(a), device=ctx.device)  # noqa: E731
    b, info = model.bdraw(dev(ph), C, z=dev(z))
    b = b.cpu().numpy()
    assert not info.cpu().numpy().any()
    order = O.chol_order(m, d["fidx"])
    for c in range(C):
        phi = np.full(m, 1e-40)
        phi[d["fidx"]] = ph[c]
        bx = exact_chol_draw(T, N, r, phi, z[c, :m], order)
        assert normwise_rel(b[c, :m], bx) < 1e-9, (n_f, c, normwise_rel(b[c, :m], bx))
    # device Philox draws: finite, and mean-zero noise around the z = 0 draw
    bp, infop = model.bdraw(dev(ph), C)
    assert np.isfinite(bp.cpu().numpy()).all() and not infop.cpu().numpy().any()


def test_big_bdraw_flags_non_positive_definite(ctx):
    import torch
    from pulsar_timing_gibbsspec_amd import synthetic
    from pulsar_timing_gibbsspec_amd.engine import DeviceModel
    d = synthetic.config5_array(n_psr=1, n_toa=600, n_f=100, seed=5)
    model = DeviceModel(ctx, d["T"], [d["sigma"][0] ** 2], d["r"], [d["fidx"]], [d["phiinv_fixed"]])
    ph = np.full((2, 200), 1e10)
    ph[1, 37] = -1e30          # column 37 of system 1 is not positive definite
    _, info = model.bdraw(torch.as_tensor(ph, device=ctx.device), 2)
    info = info.cpu().numpy()
    assert info[0] == 0 and info[1] > 0


@pytest.mark.parametrize("n_tm,n_toa", [(16, 700), (15, 700), (15, 701)])
def test_syrk_tnt_per_system(ctx, n_tm, n_toa):
    """gs_white_tnt (batched SYRK, augmented r column) == numpy TNT/d for every
    (pulsar, chain) system at m = 216, x one row per system (GS_OPT_X_PER_SYS).  T reaches LDS by
    LDS-DMA in 16-byte units when every row starts 16-byte aligned (m = 216), else in 4-byte units
    (m = 215; with 701 TOAs the second pulsar's rows start at odd offsets too), and the last chunk is
    partial (700 = 21 x 32 + 28)."""
    import torch
    from pulsar_timing_gibbsspec_amd import _lib, synthetic
    from pulsar_timing_gibbsspec_amd.white import WhiteNoiseModel
    d = synthetic.config5_array(n_psr=2, n_toa=n_toa, n_f=100, n_tm=n_tm, seed=6)
    C = 3
    c2 = _lib.Context(0, seed=1)
    c2.set_option(_lib.OPT_X_PER_SYS, 1)
    wm = WhiteNoiseModel(c2, d["T"], d["r"], d["sigma"], d["backend"], [d["fidx"]] * 2,
                         [d["phiinv_fixed"]] * 2, [d["white"]] * 2, C)
    rng = np.random.default_rng(7)
    x = np.repeat(d["x0"], C, axis=0)
    for col, kind, k, lo, hi in d["white"]:
        x[:, col] = rng.uniform(lo, hi, 2 * C)
    wm.refresh(torch.as_tensor(x, device=c2.device), d["n_param"])
    for p in range(2):
        for c in range(C):
            N = _white_N(d, p, x[p * C + c])
            TNT, dd = O.tnt(d["T"][p], N, d["r"][p])
            TNTd, ddd = wm.tnt_host(p, c)
            assert np.max(np.abs(TNTd - TNT)) <= 1e-12 * np.max(np.abs(TNT))
            assert normwise_rel(ddd, dd) < 1e-12
    assert int(wm.pinfo.abs().sum()) == 0


@pytest.mark.parametrize("n_f", [30, 100])
def test_array_engine_equals_single_pulsar_engines(n_f):
    """P independent pulsars x C chains in one WhiteArrayChains == P single-pulsar
    WhiteFreeSpectrumChains (each pinned to the reference in test_gpu_white.py) fed the
    same injected draws: bit-identical x and b after every sweep."""
    import torch
    from pulsar_timing_gibbsspec_amd import _lib, synthetic
    from pulsar_timing_gibbsspec_amd.white import WhiteArrayChains, WhiteFreeSpectrumChains, WhiteNoiseModel
    if not gpu_available():
        pytest.skip("no GPU")
    P, C, K, acl = 3, 2, 3, 6
    d = synthetic.config5_array(n_psr=P, n_toa=500, n_f=n_f, seed=8)
    n_param, NF = d["n_param"], 2 * n_f
    rng = np.random.default_rng(9)
    m = d["T"][0].shape[1]
    ctx_a = _lib.Context(0, seed=2)
    wm = WhiteNoiseModel(ctx_a, d["T"], d["r"], d["sigma"], d["backend"], [d["fidx"]] * P,
                         [d["phiinv_fixed"]] * P, [d["white"]] * P, C)
    x0 = np.repeat(d["x0"], C, axis=0)
    eng = WhiteArrayChains(wm, n_param, d["gw_cols"], d["rhomin"], d["rhomax"], x0, aclength=acl)
    dev = ctx_a.device
    ldb = wm.ldb
    z0 = np.zeros((P * C, ldb))
    z0[:, :m] = rng.standard_normal((P * C, m))
    zs = np.zeros((K, P * C, ldb))
    zs[:, :, :m] = rng.standard_normal((K, P * C, m))
    us = rng.random((K, P * C, n_f))
    nw = len(d["white"])
    mh = np.stack([rng.choice([0.1, 0.5, 1.0, 3.0, 10.0], (K, acl, P * C)),
                   rng.integers(0, nw, (K, acl, P * C)).astype(float),
                   rng.standard_normal((K, acl, P * C)), rng.random((K, acl, P * C))], axis=-1)
    T_ = lambda a: torch.as_tensor(np.ascontiguousarray(a), device=dev)  # noqa: E731
    xa, ba = [], []
    for ii in range(K):
        eng.sweep(z0=T_(z0) if ii == 0 else None, z=T_(zs[ii]), u=T_(us[ii]), mh_inj=T_(mh[ii]))
        xa.append(eng.x.cpu().numpy().copy())
        ba.append(eng.b.cpu().numpy().copy())
    for p in range(P):
        ctx_s = _lib.Context(0, seed=2)
        w1 = WhiteNoiseModel(ctx_s, [d["T"][p]], [d["r"][p]], [d["sigma"][p]], [d["backend"][p]], [d["fidx"]],
                             [d["phiinv_fixed"]], [d["white"]], C)
        s1 = WhiteFreeSpectrumChains(w1, n_param, d["gw_cols"], d["rhomin"], d["rhomax"], x0[p * C:(p + 1) * C],
                                     aclength=acl)
        sl = slice(p * C, (p + 1) * C)
        for ii in range(K):
            s1.sweep(z0=T_(z0[sl]) if ii == 0 else None, z=T_(zs[ii][sl]), u=T_(us[ii][sl]),
                     mh_inj=T_(mh[ii][:, sl]))
            assert np.array_equal(s1.x.cpu().numpy(), xa[ii][sl]), (p, ii)
            assert np.array_equal(s1.b.cpu().numpy()[:, :m], ba[ii][sl, :m]), (p, ii)
    assert int(eng.info.abs().sum()) == 0
    assert NF == 2 * n_f


def test_array_engine_philox_runs(ctx):
    """Device-RNG sweeps of the array engine: finite state, every system moves."""
    from pulsar_timing_gibbsspec_amd import _lib, synthetic
    from pulsar_timing_gibbsspec_amd.white import WhiteArrayChains, WhiteNoiseModel
    P, C = 4, 3
    d = synthetic.config5_array(n_psr=P, n_toa=800, n_f=100, seed=12)
    c3 = _lib.Context(0, seed=3)
    wm = WhiteNoiseModel(c3, d["T"], d["r"], d["sigma"], d["backend"], [d["fidx"]] * P,
                         [d["phiinv_fixed"]] * P, [d["white"]] * P, C)
    eng = WhiteArrayChains(wm, d["n_param"], d["gw_cols"], d["rhomin"], d["rhomax"],
                           np.repeat(d["x0"], C, axis=0), aclength=10)
    x0 = eng.x.cpu().numpy().copy()
    for _ in range(5):
        eng.sweep()
    x = eng.x.cpu().numpy()
    assert np.isfinite(x).all() and np.isfinite(eng.b.cpu().numpy()).all()
    assert (np.abs(x - x0).sum(axis=1) > 0).all()
    assert int(eng.info.abs().sum()) == 0
    gw = d["gw_cols"]
    assert (x[:, gw] >= -9.0).all() and (x[:, gw] <= -4.0).all()


def test_full_size_config4_pulsar(ctx):
    """One pulsar of BASELINE configs[4] at its full size (10^4 TOAs, 4 backends, n_f = 100,
    m = 216): the per-chain batched SYRK against numpy's TNT/d and the b draw against the
    exact long-double Cholesky draw with the same normals (the bench runs 200 of these)."""
    import torch
    from pulsar_timing_gibbsspec_amd import _lib, synthetic
    from pulsar_timing_gibbsspec_amd.engine import DeviceModel
    from pulsar_timing_gibbsspec_amd.white import WhiteNoiseModel
    d = synthetic.config5_array(n_psr=1, n_toa=10000, n_f=100, seed=21)
    T, r = d["T"][0], d["r"][0]
    assert T.shape == (10000, 216)
    C = 2
    c2 = _lib.Context(0, seed=2)
    c2.set_option(_lib.OPT_X_PER_SYS, 1)
    wm = WhiteNoiseModel(c2, d["T"], d["r"], d["sigma"], d["backend"], [d["fidx"]], [d["phiinv_fixed"]],
                         [d["white"]], C)
    rng = np.random.default_rng(22)
    x = np.repeat(d["x0"], C, axis=0)
    for col, kind, k, lo, hi in d["white"]:
        x[:, col] = rng.uniform(lo, hi, C)
    wm.refresh(torch.as_tensor(x, device=c2.device), d["n_param"])
    for c in range(C):
        TNT, dd = O.tnt(T, _white_N(d, 0, x[c]), r)
        TNTd, ddd = wm.tnt_host(0, c)
        assert np.max(np.abs(TNTd - TNT)) <= 1e-12 * np.max(np.abs(TNT))
        assert normwise_rel(ddd, dd) < 1e-12
    # b draw at the full size, fixed white noise (sigma^2), injected normals
    N = d["sigma"][0] ** 2
    model = DeviceModel(ctx, [T], [N], [r], [d["fidx"]], [d["phiinv_fixed"]])
    m = T.shape[1]
    logrho = rng.uniform(-8.5, -5.0, (1, 100))
    ph = 1.0 / np.repeat(10 ** (2 * logrho), 2, axis=1)
    z = np.zeros((1, model.ldb))
    z[:, :m] = rng.standard_normal((1, m))
    dev = lambda a: torch.as_tensor(np.ascontiguousarray(a), device=ctx.device)  # noqa: E731
    b, info = model.bdraw(dev(ph), 1, z=dev(z))
    assert not info.cpu().numpy().any()
    phi = np.full(m, 1e-40)
    phi[d["fidx"]] = ph[0]
    order = O.chol_order(m, d["fidx"])
    bx = exact_chol_draw(T, N, r, phi, z[0, :m], order)
    # numpy's own fp64 draw (cond(S) ~ 1e11 at 10^4 TOAs), for comparison
    # (blocked dgemm TNT, LAPACK Cholesky, the same normals) against the exact draw
    import scipy.linalg as sl
    S = (T.T @ (T / N[:, None]) + np.diag(phi))[np.ix_(order, order)]
    L = np.linalg.cholesky(S)
    y = sl.solve_triangular(L, (T.T @ (r / N))[order], lower=True) + z[0, order]
    bn = np.empty(m)
    bn[order] = sl.solve_triangular(L.T, y, lower=False)
    floor = normwise_rel(bn, bx)
    err = normwise_rel(b.cpu().numpy()[0, :m], bx)
    # double-double TNT + prefix: measured 1.5e-11 on MI355X, numpy 7.3e-10
    assert err < 1e-10 and err < floor, (err, floor)
