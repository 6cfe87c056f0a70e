"""Any number of free-spectrum bins and timing-model columns (model_definition.py:21, 66,
207: ``common_components`` is any n_f; :185-189: ``tm_marg`` gives no timing-model
columns in T).

The register-tile b draw and the fused sweep take any even NF = 2 n_f <= 64 (one
instantiation per tile count, NF at run time; 20 / 40 / 60 keep their tuned fixed-NF
builds); NF > 64 runs the workspace-tile draw in a per-sweep launch sequence with the same
Philox counters.  nm = 0 (no fixed-prior block) and up to 64 timing-model columns.

Oracles: the exact long-double Cholesky draw with the same normals (1e-9 normwise), the
oracle's Cholesky sweep loop on the same injected normals / uniforms (1e-9), and the
marginalised likelihood of pulsar_gibbs.py:569-610 (1e-10 relative).  Timing models of 70..128
columns (DMX-like windows, synthetic.synthetic_design_matrix) exercise gs_prefix's wide kernel
and gs_bdraw's wide draw (z_M rows >= 64 from Philox slot 64 + lane)."""
import numpy as np
import pytest

from oracle import gibbs_oracle as O
from tests.parity_data import exact_chol_draw_pre, exact_tnt, normwise_rel

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def ctx():
    from pulsar_timing_gibbsspec_amd import _lib
    return _lib.Context(0, seed=99)


def _pulsar(n_f, nm):
    from pulsar_timing_gibbsspec_amd import synthetic
    pta = synthetic.single_pulsar_pta("J1713+0747", n_f=n_f, tm_cols=nm, seed=2)
    return pta.get_basis()[0], pta.get_ndiag({})[0], pta.get_residuals()[0]


def _model(ctx, n_f, nm):
    from pulsar_timing_gibbsspec_amd.engine import DeviceModel
    T, N, r = _pulsar(n_f, nm)
    return DeviceModel(ctx, [T], [N], [r], [np.arange(2 * n_f)], [np.full(nm, 1e-40)]), T, N, r


def dev(a):
    return torch.as_tensor(np.ascontiguousarray(a), dtype=torch.float64).cuda()


@pytest.mark.parametrize("n_f,nm", [(1, 16), (7, 0), (7, 16), (15, 16), (16, 8), (23, 0), (31, 16), (32, 16),
                                    (40, 16), (15, 100), (30, 128), (32, 70)])
def test_bdraw_any_nf_matches_exact_draw(ctx, n_f, nm):
    model, T, N, r = _model(ctx, n_f, nm)
    m = T.shape[1]
    rng = np.random.default_rng(n_f + 100 * nm)
    C = 4
    logrho = rng.uniform(-8.5, -5.0, (C, n_f))
    ph = 1.0 / np.repeat(10 ** (2 * logrho), 2, axis=1)
    z = np.zeros((C, model.ldb))
    z[:, :m] = rng.standard_normal((C, m))
    b, info = model.bdraw(dev(ph), C, z=dev(z))
    b = b.cpu().numpy()
    assert not info.cpu().numpy().any()
    tl = exact_tnt(T, N, r)
    order = O.chol_order(m, np.arange(2 * n_f))
    for c in range(C):
        phi = np.concatenate([ph[c], np.full(nm, 1e-40)])
        bx = exact_chol_draw_pre(tl, phi, z[c, :m], order)
        assert normwise_rel(b[c, :m], bx) < 1e-9, (n_f, nm, c, normwise_rel(b[c, :m], bx))


@pytest.mark.parametrize("n_f,nm", [(7, 16), (15, 0), (15, 16), (32, 16), (40, 16), (30, 100)])
def test_sweep_any_nf_matches_oracle_loop(ctx, n_f, nm):
    """FreeSpectrumChains (fused for NF <= 64, launch sequence above) == the oracle's
    PulsarBlockGibbs loop (pulsar_gibbs.py:656-698) with the Cholesky draw on the same draws."""
    from pulsar_timing_gibbsspec_amd.engine import FreeSpectrumChains
    model, T, N, r = _model(ctx, n_f, nm)
    m = T.shape[1]
    n, C = 20, 3
    rng = np.random.default_rng(7 * n_f + nm)
    x0 = rng.uniform(-9, -4, (C, n_f))
    z = np.zeros((n + 1, C, model.ldb))
    z[:, :, :m] = rng.standard_normal((n + 1, C, m))
    U = rng.random((n, C, n_f))
    run = FreeSpectrumChains(model, 1e-18, 1e-8, C, x0)
    assert run.fused == (2 * n_f <= 64 and nm <= 64)
    xr, br = run.run(n, z0_inj=dev(z[0]), z_inj=dev(z[1:]), u_inj=dev(U))
    xr, br = xr.cpu().numpy(), br.cpu().numpy()
    assert not run.info.cpu().numpy().any()
    TNT, d = O.tnt(T, N, r)
    order = O.chol_order(m, np.arange(2 * n_f))
    tl = exact_tnt(T, N, r)
    for c in range(C):
        want_x, want_b, _ = O.sweep_single(TNT, d, np.arange(2 * n_f), x0[c], 1e-18, 1e-8, z[:, c, :m], U[:, c], n,
                                           lambda x: O.phiinv_single(x, nm), draw="chol", order=order)
        assert normwise_rel(xr[:, c], want_x) < 1e-9, (n_f, nm, c)
        # b: each draw against the exact draw at the device's own state (a fed-back b chain
        # amplifies 1e-10 rounding through phi = 10^(2x); see tests/test_gpu_indep.py)
        assert normwise_rel(br[1, c, :m], want_b[1]) < 1e-9, (n_f, nm, c)
        for j in range(1, n):
            bx = exact_chol_draw_pre(tl, O.phiinv_single(xr[j, c], nm), z[j, c, :m], order)
            assert normwise_rel(br[j, c, :m], bx) < 1e-9, (n_f, nm, c, j)


@pytest.mark.parametrize("n_f,nm", [(7, 16), (15, 0), (32, 16), (30, 48), (30, 64), (30, 100)])
def test_lnlike_marg_any_nf(ctx, n_f, nm):
    model, T, N, r = _model(ctx, n_f, nm)
    rng = np.random.default_rng(n_f)
    C = 3
    logrho = rng.uniform(-8.5, -5.0, (C, n_f))
    ph = 1.0 / np.repeat(10 ** (2 * logrho), 2, axis=1)
    lnl, info = model.lnlike_marg(dev(ph), C)
    lnl = lnl.cpu().numpy()
    assert not info.cpu().numpy().any()
    TNT, d = O.tnt(T, N, r)
    for c in range(C):
        phi = np.concatenate([1.0 / ph[c], np.full(nm, 1e40)])
        want = O.lnlike_fullmarg(r, N, TNT, d, 1.0 / phi, np.sum(np.log(phi)))
        assert abs(lnl[c] - want) <= 1e-10 * abs(want), (n_f, nm, c, lnl[c], want)


def test_pulsar_block_gibbs_with_15_bins_and_no_timing_model(tmp_path):
    """The drop-in with common_components = 15 and a marginalised timing model (nm = 0)."""
    from pulsar_timing_gibbsspec_amd import PulsarBlockGibbs, synthetic
    pta = synthetic.single_pulsar_pta("J1713+0747", n_f=15, tm_cols=0, seed=4)
    gb = PulsarBlockGibbs(pta, seed=3, nchains=8)
    x0 = np.random.default_rng(0).uniform(-9, -4, 15)
    chain = gb.sample(x0, outdir=str(tmp_path), niter=150)
    assert chain.shape == (150, 15) and gb.bchain.shape == (150, 30)
    assert np.all(np.isfinite(gb.chains)) and gb.chains.min() >= -9 and gb.chains.max() <= -4
    assert np.load(tmp_path / "chain.npy").shape == (101, 15)


def test_big_nf_non_pd_keeps_b(ctx):
    """The workspace-tile draw (NF > 64): a non-PD system keeps its previous b and is flagged."""
    model, T, N, r = _model(ctx, 40, 16)
    assert model.NF == 80
    rng = np.random.default_rng(4)
    ph = np.full((2, 80), 1e12)
    ph[0] = -1e30
    prev = rng.standard_normal((2, model.ldb))
    b, info = model.bdraw(dev(ph), 2, z=dev(rng.standard_normal((2, model.ldb))), out=dev(prev))
    b, info = b.cpu().numpy(), info.cpu().numpy()
    assert info[0] > 0 and info[1] == 0
    assert np.array_equal(b[0], prev[0]) and np.all(np.isfinite(b[1])) and not np.array_equal(b[1], prev[1])


@pytest.mark.parametrize("sched", [0, 1])
def test_sweep_nmx64_4096_chains_falls_back_to_4_wave(ctx, sched):
    """NF = 60 with a 64-column timing model at 4096 chains: the 12-wave hand-off workgroup would
    need 168 KB of LDS (> 160 KB), so the launcher must run the 4-wave shape even when the cost
    model (sched 0) or GS_OPT_SWEEP_SCHED = 1 asks for hand-off workgroups.  Same
    draws: bit for bit the chains of GS_OPT_SWEEP_SCHED = 2; chains 0 and 4095 equal the oracle's
    Cholesky loop on the injected normals / uniforms (1e-9) and every draw is the exact draw."""
    from pulsar_timing_gibbsspec_amd import _lib
    from pulsar_timing_gibbsspec_amd.engine import FreeSpectrumChains
    model, T, N, r = _model(ctx, 30, 64)
    assert model.NMX == 64
    m = T.shape[1]
    C, S = 4096, 4
    rng = np.random.default_rng(5)
    x0 = rng.uniform(-9, -5, (C, 30))
    z = np.zeros((S + 1, C, model.ldb))
    z[:, :, :m] = rng.standard_normal((S + 1, C, m))
    U = rng.random((S, C, 30))
    zd0, zd, Ud = dev(z[0]), dev(z[1:]), dev(U)
    out = []
    prev = ctx.get_option(_lib.OPT_SWEEP_SCHED)
    try:
        for sc in (sched, 2):
            ctx.set_option(_lib.OPT_SWEEP_SCHED, sc)
            run = FreeSpectrumChains(model, 1e-18, 1e-8, C, x0)
            xr, br = run.run(S, z0_inj=zd0, z_inj=zd, u_inj=Ud)
            run.check_info()
            out.append([t.cpu().numpy() for t in (xr, br, run.x, run.b, run.info)])
    finally:
        ctx.set_option(_lib.OPT_SWEEP_SCHED, prev)
    for a, b in zip(*out):
        assert np.array_equal(a, b)
    assert not out[0][-1].any()
    xr, br = out[0][0], out[0][1]
    TNT, d = O.tnt(T, N, r)
    order = O.chol_order(m, np.arange(60))
    tl = exact_tnt(T, N, r)
    for c in (0, C - 1):
        want_x, _, _ = O.sweep_single(TNT, d, np.arange(60), x0[c], 1e-18, 1e-8, z[:, c, :m], U[:, c], S,
                                      lambda x: O.phiinv_single(x, 64), draw="chol", order=order)
        assert normwise_rel(xr[:, c], want_x) < 1e-9, c
        for j in range(1, S):
            bx = exact_chol_draw_pre(tl, O.phiinv_single(xr[j, c], 64), z[j, c, :m], order)
            assert normwise_rel(br[j, c, :m], bx) < 1e-9, (c, j)
