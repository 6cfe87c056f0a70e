"""HIP path vs the oracle / the reference's golden vectors (needs an MI355X).

Tolerances: integer work (Philox words) bit-exact; fp64 draws within 1e-9
relative, norm-wise per draw (north_star: "within 1e-9 relative in fp64");
posteriors: two-sample KS per frequency bin against a long reference chain.
"""
import numpy as np
import pytest

from oracle import gibbs_oracle as O
from tests.conftest import golden
from tests.parity_data import normwise_rel, single_replay

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def ctx():
    from pulsar_timing_gibbsspec_amd import _lib
    return _lib.Context(0, seed=1234)


@pytest.fixture(scope="module")
def replay():
    return single_replay(golden("single_j1713.npz"))


@pytest.fixture(scope="module")
def model(ctx):
    from pulsar_timing_gibbsspec_amd.engine import DeviceModel
    g = golden("single_j1713.npz")
    gwid = np.asarray(g["gwid"])
    n_tm = g["T"].shape[1] - gwid.size
    return DeviceModel(ctx, [g["T"]], [g["Nvec"]], [g["r"]], [gwid], [np.full(n_tm, 1e-40)])


@pytest.fixture(scope="module")
def exact_chain(replay):
    """The J1713 fixture run replayed with every b draw exact (long double): what an error-free
    b|rho does on the reference's draws.  Its fed-back b is 1.06e-9 from the reference's own
    bchain after 300 sweeps (tools/closed_loop_ref.py: the reference's per-draw fp64 error,
    <= 8.8e-11, amplified through rho), x stays within 4e-11."""
    from tests.parity_data import exact_sweep_single, exact_tnt
    g = golden("single_j1713.npz")
    tl = exact_tnt(g["T"], g["Nvec"], g["r"])
    return exact_sweep_single(tl, replay["gwid"], g["x0"], replay["rhomin"], replay["rhomax"], replay["zc"],
                              g["U"], replay["niter"], lambda x: O.phiinv_single(x, replay["n_tm"]),
                              replay["order"]), tl


def dev(a, dtype=torch.float64):
    return torch.as_tensor(np.ascontiguousarray(a), dtype=dtype).cuda()


def test_philox_bitexact(ctx):
    from pulsar_timing_gibbsspec_amd import _lib
    rng = np.random.default_rng(0)
    ctr = rng.integers(0, 2 ** 32, size=(4096, 4), dtype=np.uint64).astype(np.uint32)
    out = torch.zeros(4096, 4, dtype=torch.int32, device="cuda")
    c = dev(ctr.view(np.int32), torch.int32)
    _lib.check(ctx.lib.gs_philox(ctx.handle, 4096, _lib.ptr(c), _lib.ptr(out)), "gs_philox")
    got = out.cpu().numpy().view(np.uint32)
    key = np.array([[1234 & 0xffffffff, 1234 >> 32]], np.uint32)
    want = O.philox4x32(ctr, np.repeat(key, 4096, axis=0))
    assert np.array_equal(got, want)


def test_tnt_matches_numpy(model, replay):
    TNT, d = model.tnt_host(0)
    assert normwise_rel(TNT, replay["TNT"]) < 1e-12
    assert normwise_rel(d, replay["d"]) < 1e-12


def test_tnt_dd_and_prefix_dd_accuracy(model):
    """gs_tnt_dd: TNT + TNT_lo against the long-double TNT of the same fp64 inputs; gs_prefix_dd:
    S0 and dF against a long-double prefix of that TNT."""
    from tests.parity_data import exact_tnt
    g = golden("single_j1713.npz")
    tl = exact_tnt(g["T"], g["Nvec"], g["r"])
    m = g["T"].shape[1]
    L_ = np.longdouble
    hi = model.TNT.cpu().numpy().reshape(m, m).astype(L_) + model.TNT_lo.cpu().numpy().reshape(m, m)
    scale = float(np.max(np.abs(np.asarray(tl[0], np.float64))))
    assert float(np.max(np.abs(hi - tl[0]))) / scale < 2e-17
    dd = model.d.cpu().numpy().astype(L_) + model.d_lo.cpu().numpy()
    assert float(np.max(np.abs(dd - tl[1]))) / float(np.max(np.abs(np.asarray(tl[1], np.float64)))) < 2e-17
    assert np.array_equal(model.TNT.cpu().numpy().reshape(m, m), model.TNT.cpu().numpy().reshape(m, m).T)
    gwid = np.asarray(g["gwid"])
    order = O.chol_order(m, gwid)
    Mi, Fi = order[:m - gwid.size], order[m - gwid.size:]
    A = tl[0].copy()
    A[Mi, Mi] += L_(1e-40)
    AMM = A[np.ix_(Mi, Mi)]
    nm = Mi.size
    LM = np.zeros_like(AMM)
    for k in range(nm):
        v = AMM[k:, k] - LM[k:, :k] @ LM[k, :k]
        LM[k, k] = np.sqrt(v[0])
        LM[k + 1:, k] = v[1:] / LM[k, k]
    W = np.zeros((nm, Fi.size + 1), dtype=L_)
    B = np.concatenate([A[np.ix_(Mi, Fi)], tl[1][Mi][:, None]], axis=1)
    for i in range(nm):
        W[i] = (B[i] - LM[i, :i] @ W[:i]) / LM[i, i]
    S0x = np.asarray(A[np.ix_(Fi, Fi)] - W[:, :-1].T @ W[:, :-1], np.float64)
    dFx = np.asarray(tl[1][Fi] - W[:, :-1].T @ W[:, -1], np.float64)
    NF = model.NF
    buf = model.model.cpu().numpy()
    S0 = buf[: NF * (NF + 1)].reshape(NF, NF + 1)[:, :NF]
    dF = buf[NF * (NF + 1): NF * (NF + 1) + NF]
    assert normwise_rel(S0, S0x) < 1e-15
    assert normwise_rel(dF, dFx) < 1e-15
    assert np.array_equal(S0, S0.T)


def test_prefix_matches_oracle(model, replay):
    NF, NMX = model.NF, model.NMX
    pf = O.prefix_factor(replay["TNT"], replay["d"], replay["gwid"], np.full(replay["n_tm"], 1e-40))
    buf = model.model.cpu().numpy()
    S0 = buf[: NF * (NF + 1)].reshape(NF, NF + 1)[:, :NF]
    o = NF * (NF + 1)
    dF = buf[o:o + NF]
    o += NF
    G = buf[o:o + NMX * (NF + 1)].reshape(NMX, NF + 1)[:, :NF]
    o += NMX * (NF + 1)
    h = buf[o:o + NMX]
    o += NMX
    R = buf[o:o + NMX * NMX].reshape(NMX, NMX)
    assert normwise_rel(S0, pf["S0"]) < 1e-9
    assert normwise_rel(dF, pf["dF"]) < 1e-9
    assert normwise_rel(G, pf["G"]) < 1e-9
    assert normwise_rel(h, pf["h"]) < 1e-9
    assert normwise_rel(R, pf["R"]) < 1e-9


@pytest.mark.parametrize("bcast", [0, 1, 2, 3])
def test_bdraw_matches_reference_draws(ctx, model, replay, bcast):
    """gs_bdraw with rotated normals == the reference's SVD draw (1e-9)."""
    from pulsar_timing_gibbsspec_amd import _lib
    ctx.set_option(_lib.OPT_BCAST, bcast)
    g = golden("single_j1713.npz")
    ks = list(range(replay["niter"] + 1))          # every draw of the reference's run (open loop)
    ph = np.stack([replay["phiinv"][k][replay["gwid"]] for k in ks])
    z = np.stack([replay["zc"][k] for k in ks])
    # one pulsar, len(ks) chains: system c uses row c
    b, info = model.bdraw(dev(ph), len(ks), z=dev(z))
    b = b.cpu().numpy()
    assert not info.cpu().numpy().any()
    for c, k in enumerate(ks):
        b_ref = O.bdraw_svd(replay["TNT"], replay["d"], replay["phiinv"][k], g["z"][k])
        assert normwise_rel(b[c], b_ref) < 1e-9, k
    ctx.set_option(_lib.OPT_BCAST, 3)


def test_bdraw_flags_non_positive_definite(model):
    """A non-PD system (negative prior precision) is flagged in info and keeps its previous b
    (the reference's LinAlgError branch, pulsar_gibbs.py:507-516): no NaN reaches the state;
    the other systems of the batch draw normally; an attached counter counts the failure."""
    from pulsar_timing_gibbsspec_amd.engine import fail_counts
    rng = np.random.default_rng(3)
    C = 3
    ph = np.full((C, model.NF), 1e12)
    ph[1] = -1e30                               # system 1: indefinite
    prev = rng.standard_normal((C, model.ldb))
    out = dev(prev)
    cnt = torch.zeros(C, dtype=torch.int32, device="cuda")
    with fail_counts(model.ctx, cnt):
        b, info = model.bdraw(dev(ph), C, z=dev(rng.standard_normal((C, model.ldb))), out=out)
    b, info = b.cpu().numpy(), info.cpu().numpy()
    assert info[1] > 0 and info[0] == 0 and info[2] == 0
    assert np.array_equal(b[1], prev[1])
    assert np.all(np.isfinite(b)) and not np.array_equal(b[0], prev[0])
    assert cnt.cpu().tolist() == [0, 1, 0]


@pytest.mark.parametrize("sched", [2, 3])
def test_fused_sweep_non_pd_mid_run_keeps_b(ctx, model, replay, sched):
    """k_sweep_freespec (sched 2) and k_sweep_pair (sched 3) with Sigma made indefinite mid-run (the
    model block's S0[0][0] set to -1e300 after 10 sweeps): the failing draws keep each chain's
    previous b (never NaN), the rho|b step goes on, every failure is counted as it happens, and once
    the model is restored the chains draw again."""
    from pulsar_timing_gibbsspec_amd import _lib
    from pulsar_timing_gibbsspec_amd.engine import FreeSpectrumChains
    g = golden("single_j1713.npz")
    C = 4
    prev = ctx.get_option(_lib.OPT_SWEEP_SCHED)
    ctx.set_option(_lib.OPT_SWEEP_SCHED, sched)
    run = FreeSpectrumChains(model, replay["rhomin"], replay["rhomax"], C, g["x0"])
    run.run(10)
    assert ctx.get_option(_lib.OPT_LAST_SWEEP_SHAPE) == sched
    b10 = run.b.clone()
    saved = model.model.clone()
    try:
        model.model[0] = -1e300
        xr, br = run.run(5)
        assert torch.equal(run.b, b10)                       # b kept through 5 failed draws
        assert torch.isfinite(xr).all() and torch.isfinite(br).all() and torch.isfinite(run.x).all()
        assert not torch.equal(xr[0], xr[-1])                # rho|b kept sampling
        assert (run.info.cpu().numpy() > 0).all()
        assert run.fail_count.cpu().tolist() == [5] * C
    finally:
        model.model.copy_(saved)
        ctx.set_option(_lib.OPT_SWEEP_SCHED, prev)
    ctx.set_option(_lib.OPT_SWEEP_SCHED, sched)
    run.run(5)
    ctx.set_option(_lib.OPT_SWEEP_SCHED, prev)
    assert run.fail_count.cpu().tolist() == [5] * C
    assert torch.isfinite(run.b).all() and not torch.equal(run.b, b10)


@pytest.mark.parametrize("bcast", [0, 1, 2, 3])
def test_fused_sweep_matches_reference_chain(ctx, model, replay, exact_chain, bcast):
    """gs_sweep_freespec with the reference's draws (rotated), any broadcast variant of the
    factorisation, 300 fed-back sweeps: x within 1e-9 of the reference's chain; b within 1e-9
    of the error-free replay of the same draws (the reference's own fed-back b is 1.06e-9 from
    that replay; every draw against the reference's b is test_bdraw_matches_reference_draws)."""
    from pulsar_timing_gibbsspec_amd import _lib
    from pulsar_timing_gibbsspec_amd.engine import FreeSpectrumChains
    ctx.set_option(_lib.OPT_BCAST, bcast)
    g = golden("single_j1713.npz")
    n = replay["niter"]
    nc = 3                                       # identical replicas: batch independence
    run = FreeSpectrumChains(model, replay["rhomin"], replay["rhomax"], nc, g["x0"])
    zc = replay["zc"]
    z0 = np.repeat(zc[0][None], nc, axis=0)
    zi = np.repeat(zc[1:][:, None, :], nc, axis=1)
    ui = np.repeat(g["U"][:, None, :], nc, axis=1)
    xr, br = run.run(n, z0_inj=dev(z0), z_inj=dev(zi), u_inj=dev(ui))
    xr, br = xr.cpu().numpy(), br.cpu().numpy()
    assert not run.info.cpu().numpy().any()
    (ex_x, ex_b, ex_final), _ = exact_chain
    for c in range(nc):
        assert normwise_rel(xr[:, c], g["chain"]) < 1e-9
        assert normwise_rel(xr[:, c], ex_x) < 1e-9
        assert normwise_rel(br[1:, c], ex_b[1:]) < 1e-9
        assert np.all(br[0, c] == 0)
    assert normwise_rel(run.b.cpu().numpy()[0], ex_final) < 1e-9
    assert np.array_equal(xr[:, 0], xr[:, 1]) and np.array_equal(br[:, 0], br[:, 2])
    ctx.set_option(_lib.OPT_BCAST, 3)


def test_sweep_split_and_sharding_invariance(model, replay):
    """Counter-based RNG: (a) 20 sweeps == 7 + 13 sweeps; (b) chains [4, 8) run
    alone with chain_base=4 reproduce chains 4..7 of an 8-chain run (sharding)."""
    from pulsar_timing_gibbsspec_amd.engine import FreeSpectrumChains
    g = golden("single_j1713.npz")
    a = FreeSpectrumChains(model, replay["rhomin"], replay["rhomax"], 8, g["x0"])
    xa, ba = a.run(20)
    b = FreeSpectrumChains(model, replay["rhomin"], replay["rhomax"], 8, g["x0"])
    x1, _ = b.run(7)
    x2, _ = b.run(13)
    assert torch.equal(torch.cat([x1, x2]), xa)
    c = FreeSpectrumChains(model, replay["rhomin"], replay["rhomax"], 4, g["x0"], chain_base=4)
    xc, bc = c.run(20)
    assert torch.equal(xc, xa[:, 4:8]) and torch.equal(bc, ba[:, 4:8])
    assert not torch.equal(xa[:, 0], xa[:, 1])


def test_rho_analytic_kernel(ctx, model):
    from pulsar_timing_gibbsspec_amd import _lib
    g = golden("single_j1713.npz")
    ii = np.arange(1, 299)
    b = dev(g["bchain"][ii])
    u = dev(g["U"][ii])
    x = torch.empty(ii.size, 30, dtype=torch.float64, device="cuda")
    fidx = dev(np.asarray(g["gwid"], np.int32)[None], torch.int32)
    _lib.check(ctx.lib.gs_rho_analytic(ctx.handle, 1, ii.size, 60, 76, _lib.ptr(fidx), _lib.ptr(b),
                                       _lib.ptr(u), 0, 0, float(g["rhomin"]), float(g["rhomax"]),
                                       _lib.ptr(x), 30), "gs_rho_analytic")
    assert normwise_rel(x.cpu().numpy(), g["chain"][ii + 1]) < 1e-13


def test_posterior_ks_against_reference(model, replay):
    """Independent Philox streams: log10 rho marginals match a 40k-sweep reference
    chain (tests/golden/long_j1713.npz) under a two-sample KS test per bin."""
    from scipy.stats import ks_2samp
    from pulsar_timing_gibbsspec_amd.engine import FreeSpectrumChains
    ref = golden("long_j1713.npz")["chain"].astype(np.float64)[200:][::5]   # thin 50 sweeps
    g = golden("single_j1713.npz")
    run = FreeSpectrumChains(model, replay["rhomin"], replay["rhomax"], 4096, g["x0"])
    run.run(300, record=False)
    x = run.x.cpu().numpy()                      # one draw per independent chain
    pv = np.array([ks_2samp(x[:, k], ref[:, k]).pvalue for k in range(30)])
    assert pv.min() > 1e-4 / 30, pv               # Bonferroni over 30 bins


def test_pulsar_block_gibbs_surface(tmp_path):
    """Drop-in surface: construction, update_b parity, sample() files/layout."""
    from pulsar_timing_gibbsspec_amd import PulsarBlockGibbs, synthetic
    g = golden("single_j1713.npz")
    R = single_replay(g)
    pta = synthetic.single_pulsar_pta("J1713+0747", seed=0)
    gb = PulsarBlockGibbs(pta, seed=5)
    assert np.array_equal(gb.gwid, g["gwid"])
    assert gb.rhomin == float(g["rhomin"]) and gb.rhomax == float(g["rhomax"])
    b = gb.update_b(g["x0"], z=R["zc"][0])
    assert normwise_rel(b, O.bdraw_svd(R["TNT"], R["d"], R["phiinv"][0], g["z"][0])) < 1e-9
    gb2 = PulsarBlockGibbs(pta, seed=6, nchains=4)
    chain = gb2.sample(g["x0"], outdir=str(tmp_path), niter=250)
    assert chain.shape == (250, 30)
    assert np.load(tmp_path / "chain.npy").shape == (201, 30)
    assert np.load(tmp_path / "bchain.npy").shape == (201, 76)
    assert np.load(tmp_path / "chains.npy").shape == (4, 201, 30)
    assert np.array_equal(gb2.chain[0], g["x0"]) and np.all(gb2.bchain[0] == 0)
    assert open(tmp_path / "pars_chain.txt").read().split()[0] == "gw_log10_rho_0"
    assert np.all(np.isfinite(gb2.chain)) and np.all(gb2.chain >= -9.0) and np.all(gb2.chain <= -4.0)


def test_sample_flush_final_and_resume(tmp_path):
    """flush_final writes the trailing partial block; resume continues from
    the saved rows and reproduces the uninterrupted chain (device Philox counters are
    indexed by the global sweep)."""
    from pulsar_timing_gibbsspec_amd import PulsarBlockGibbs, synthetic
    g = golden("single_j1713.npz")
    pta = synthetic.single_pulsar_pta("J1713+0747", seed=0)
    full = PulsarBlockGibbs(pta, seed=8).sample(g["x0"], outdir=str(tmp_path / "a"), niter=260,
                                                 flush_final=True)
    assert np.load(tmp_path / "a" / "chain.npy").shape == (260, 30)
    gb = PulsarBlockGibbs(pta, seed=8)
    gb.sample(g["x0"], outdir=str(tmp_path / "b"), niter=150)          # saves rows [:101]
    assert np.load(tmp_path / "b" / "chain.npy").shape == (101, 30)
    res = PulsarBlockGibbs(pta, seed=8).sample(g["x0"], outdir=str(tmp_path / "b"), niter=260, resume=True,
                                                flush_final=True)
    assert np.array_equal(res, full)


@pytest.mark.parametrize("record_bchains", [False, True])
def test_resume_many_chains(tmp_path, record_bchains):
    """nchains > 16 (default: only chain 0's b reaches the host) or record_bchains=False: resume
    reloads every chain's rows from chains.npy (rows [:start] equal the uninterrupted run's,
    never zeros) and restarts each chain from its own x; chain 0 (the reference's chain) and,
    with every b kept, all chains continue bit for bit; without every b, chains 1.. continue
    from b | x redrawn (valid, finite, inside the prior)."""
    from pulsar_timing_gibbsspec_amd import PulsarBlockGibbs, synthetic
    g = golden("single_j1713.npz")
    pta = synthetic.single_pulsar_pta("J1713+0747", seed=0)
    nc = 20
    kw = dict(record_bchains=record_bchains)
    full = PulsarBlockGibbs(pta, seed=9, nchains=nc)
    full.sample(g["x0"], outdir=str(tmp_path / "a"), niter=260, flush_final=True, **kw)
    gb = PulsarBlockGibbs(pta, seed=9, nchains=nc)
    gb.sample(g["x0"], outdir=str(tmp_path / "b"), niter=150, **kw)          # saves rows [:101]
    res = PulsarBlockGibbs(pta, seed=9, nchains=nc)
    res.sample(g["x0"], outdir=str(tmp_path / "b"), niter=260, resume=True, flush_final=True, **kw)
    a = np.load(tmp_path / "a" / "chains.npy")
    b = np.load(tmp_path / "b" / "chains.npy")
    assert a.shape == b.shape == (nc, 260, 30)
    assert np.array_equal(b[:, :101], a[:, :101])                  # restored, not zero rows
    assert np.array_equal(b[0], a[0])                              # chain 0 bit for bit
    assert np.array_equal(np.load(tmp_path / "b" / "chain.npy"), np.load(tmp_path / "a" / "chain.npy"))
    if record_bchains:
        assert np.array_equal(b, a)
    else:
        assert np.all(np.isfinite(b)) and b.min() >= -9 and b.max() <= -4
        assert not np.array_equal(b[1:, 101:], a[1:, 101:])        # b of chains 1.. was redrawn


def test_history_straight_to_pinned_host(model, replay):
    """Zero-copy history (sample()'s default): x rows and the first K chains' b rows written
    by the kernel into pinned host memory (GS_OPT_BREC_CHAINS) equal the HBM rows of the same
    sweeps, bit for bit; the option is restored after the call."""
    from pulsar_timing_gibbsspec_amd import _lib
    from pulsar_timing_gibbsspec_amd.engine import FreeSpectrumChains
    C, n, K = 8, 30, 2
    x0 = golden("single_j1713.npz")["x0"]
    ra = FreeSpectrumChains(model, replay["rhomin"], replay["rhomax"], C, x0)
    xa, ba = ra.run(n)
    rb = FreeSpectrumChains(model, replay["rhomin"], replay["rhomax"], C, x0)
    xh = torch.empty(n, C, 30, dtype=torch.float64, pin_memory=True)
    bh = torch.empty(n, K, model.ldb, dtype=torch.float64, pin_memory=True)
    rb.run(n, x_rec=xh, b_rec=bh, record_b_chains=K)
    torch.cuda.synchronize()
    assert model.ctx.get_option(_lib.OPT_BREC_CHAINS) == 0
    assert torch.equal(xh, xa.cpu())
    assert torch.equal(bh, ba.cpu()[:, :K])
    assert torch.equal(rb.b, ra.b)


def test_capi_edge_cases_and_errors():
    """The C-ABI's empty batches and argument errors (include/pulsar_gibbs.h: 0 ok, positive =
    1-based index of the offending argument, gs_last_error has the message): an empty chain
    batch launches nothing and leaves b untouched; bad NF / ldb / NULL arrays / NULL ctx are
    reported, not launched."""
    import ctypes as C
    import torch
    from pulsar_timing_gibbsspec_amd import _lib, synthetic
    from pulsar_timing_gibbsspec_amd._lib import ptr
    from pulsar_timing_gibbsspec_amd.engine import DeviceModel
    ctx = _lib.Context(0, seed=5)
    pta = synthetic.single_pulsar_pta("J1713+0747", seed=0)
    T, N, r = pta.get_basis()[0], pta.get_ndiag({})[0], pta.get_residuals()[0]
    model = DeviceModel(ctx, [T], [N], [r], [np.arange(60)], [np.full(T.shape[1] - 60, 1e-40)])
    lib, h = ctx.lib, ctx.handle
    ph = torch.ones(2, 60, dtype=torch.float64, device=ctx.device)
    b = torch.full((2, model.ldb), 7.0, dtype=torch.float64, device=ctx.device)
    info = torch.zeros(2, dtype=torch.int32, device=ctx.device)

    def call(handle=h, n_chain=2, NF=60, ldb=model.ldb, phv=ph, out=b):
        return lib.gs_bdraw(handle, 1, n_chain, NF, model.NMX, ldb, ptr(model.model), ptr(model.fidx),
                            ptr(model.midx), ptr(model.nm_dev), ptr(phv) if phv is not None else None, None, 0,
                            _lib.EV_B, 0, None, ptr(out), ptr(info))

    assert call(n_chain=0) == 0
    torch.cuda.synchronize()
    assert bool((b == 7.0).all())
    assert call(NF=61) == 4 and b"NF" in lib.gs_last_error()
    assert call(ldb=60) == 6
    assert call(phv=None) == 7
    assert call(handle=C.c_void_p(0)) == 1
    assert call(n_chain=-1) == 2
    torch.cuda.synchronize()
    assert bool((b == 7.0).all())
    assert call() == 0 and not info.cpu().numpy().any()
    torch.cuda.synchronize()
    assert bool(torch.isfinite(b).all()) and not bool((b[:, :model.m[0]] == 7.0).any())


@pytest.mark.parametrize("C,S", [(37, 10), (16, 1), (48, 31)])
def test_sweep_handoff_workgroups_equal_one_chain_per_wave(ctx, model, replay, C, S):
    """GS_OPT_SWEEP_SCHED = 1 (12-wave workgroups: each trio of waves runs a 13th..16th chain in
    thirds of the sweeps, the chain state handed over through LDS) gives bit for bit the chains
    of GS_OPT_SWEEP_SCHED = 2 (one chain per wave): ragged chain counts (16 chains = no extra
    chain ran by a full trio; 37 = a partial workgroup), 1 sweep (empty thirds), sweep 0's first
    draw, every recorded row and the final state."""
    from pulsar_timing_gibbsspec_amd import _lib
    from pulsar_timing_gibbsspec_amd.engine import FreeSpectrumChains
    x0 = np.random.default_rng(3).uniform(-9, -5, (C, 30))
    out = []
    prev = ctx.get_option(_lib.OPT_SWEEP_SCHED)
    try:
        for sched in (1, 2):
            ctx.set_option(_lib.OPT_SWEEP_SCHED, sched)
            run = FreeSpectrumChains(model, replay["rhomin"], replay["rhomax"], C, x0)
            xr, br = run.run(S)
            xr2, br2 = run.run(S + 2)                       # a second launch continues the state
            out.append([t.cpu().numpy() for t in (xr, br, xr2, br2, run.x, run.b, run.info)])
    finally:
        ctx.set_option(_lib.OPT_SWEEP_SCHED, prev)
    for a, b in zip(*out):
        assert np.array_equal(a, b)
    assert not out[0][-1].any()


@pytest.mark.parametrize("C,S", [(2, 1), (38, 7), (64, 12)])
def test_sweep_two_chains_per_wave_equal_one_chain_per_wave(ctx, model, replay, C, S):
    """GS_OPT_SWEEP_SCHED = 3 (k_sweep_pair: two chains per wavefront, the diagonal-tile eliminations
    of both in one paired register set, gibbs_tile2.h) gives bit for bit the chains of
    GS_OPT_SWEEP_SCHED = 2: every recorded row, a continued second launch and the final state; a
    partial last workgroup (38 chains = 4 full workgroups of 8 + 3 pairs)."""
    from pulsar_timing_gibbsspec_amd import _lib
    from pulsar_timing_gibbsspec_amd.engine import FreeSpectrumChains
    x0 = np.random.default_rng(6).uniform(-9, -5, (C, 30))
    out, shapes = [], []
    prev = ctx.get_option(_lib.OPT_SWEEP_SCHED)
    try:
        for sched in (2, 3):
            ctx.set_option(_lib.OPT_SWEEP_SCHED, sched)
            run = FreeSpectrumChains(model, replay["rhomin"], replay["rhomax"], C, x0)
            xr, br = run.run(S)
            xr2, br2 = run.run(S + 3)
            shapes.append(ctx.get_option(_lib.OPT_LAST_SWEEP_SHAPE))
            out.append([t.cpu().numpy() for t in (xr, br, xr2, br2, run.x, run.b, run.info)])
    finally:
        ctx.set_option(_lib.OPT_SWEEP_SCHED, prev)
    assert shapes == [2, 3]                      # the kernels that ran: one chain per wave, two
    for a, b in zip(*out):
        assert np.array_equal(a, b)
    assert not out[1][-1].any()


def test_sweep_cost_model_shapes(ctx, model, replay):
    """GS_OPT_SWEEP_SCHED = 0: the cost model runs two chains per wave where that kernel fills its
    2 waves/SIMD (the headline's 4096 chains on a 256-CU MI355X) and the one-chain shapes where it
    would leave SIMDs with one wave (2048 chains) or needs an even chain count (4095); setting the
    read-only GS_OPT_LAST_SWEEP_SHAPE fails."""
    from pulsar_timing_gibbsspec_amd import _lib
    from pulsar_timing_gibbsspec_amd.engine import FreeSpectrumChains
    assert ctx.get_option(_lib.OPT_SWEEP_SCHED) == 0
    got = {}
    for C in (4096, 2048, 4095):
        x0 = np.random.default_rng(C).uniform(-9, -5, (C, 30))
        FreeSpectrumChains(model, replay["rhomin"], replay["rhomax"], C, x0).run(1)
        got[C] = ctx.get_option(_lib.OPT_LAST_SWEEP_SHAPE)
    if torch.cuda.get_device_properties(0).multi_processor_count == 256:
        assert got[4096] == 3
    assert got[2048] != 3 and got[4095] != 3
    with pytest.raises(RuntimeError):
        ctx.set_option(_lib.OPT_LAST_SWEEP_SHAPE, 1)


def test_sweep_handoff_timeout_fails_loudly(ctx, model, replay):
    """A hand-off that never arrives (GS_OPT_DEBUG_HANDOFF: workgroup 0's first trio does not
    publish its first third) must not be read: the extra chain (chain 12 of workgroup 0) ends with
    info = -1, its state is not advanced (x_state keeps x0, no stale row), every other chain is
    the one-chain-per-wave run's bit for bit, and FreeSpectrumChains.check_info() raises."""
    from pulsar_timing_gibbsspec_amd import _lib
    from pulsar_timing_gibbsspec_amd.engine import FreeSpectrumChains
    C, S = 32, 9
    x0 = np.random.default_rng(4).uniform(-9, -5, (C, 30))
    prev = ctx.get_option(_lib.OPT_SWEEP_SCHED)
    try:
        ctx.set_option(_lib.OPT_SWEEP_SCHED, 2)
        ref = FreeSpectrumChains(model, replay["rhomin"], replay["rhomax"], C, x0)
        ref.run(S)
        ctx.set_option(_lib.OPT_SWEEP_SCHED, 1)
        ctx.set_option(_lib.OPT_DEBUG_HANDOFF, 1)
        run = FreeSpectrumChains(model, replay["rhomin"], replay["rhomax"], C, x0)
        run.run(S)
    finally:
        ctx.set_option(_lib.OPT_DEBUG_HANDOFF, 0)
        ctx.set_option(_lib.OPT_SWEEP_SCHED, prev)
    info = run.info.cpu().numpy()
    assert info[12] == -1
    assert not np.delete(info, 12).any()
    x = run.x.cpu().numpy()
    assert np.array_equal(x[12], x0[12])                       # never advanced from a stale slot
    keep = np.delete(np.arange(C), 12)
    assert np.array_equal(x[keep], ref.x.cpu().numpy()[keep])
    assert np.array_equal(run.b.cpu().numpy()[keep], ref.b.cpu().numpy()[keep])
    with pytest.raises(RuntimeError, match="hand-off"):
        run.check_info()
    ref.check_info()


def test_fail_counts_scopes_nest(ctx):
    """engine.fail_counts restores the attachment it replaced: an inner engine's
    scope inside an outer one leaves the outer counter attached."""
    from pulsar_timing_gibbsspec_amd.engine import fail_counts
    a = torch.zeros(4, dtype=torch.int32, device=ctx.device)
    b = torch.zeros(4, dtype=torch.int32, device=ctx.device)
    assert getattr(ctx, "_fail_counts_attached", None) is None
    with fail_counts(ctx, a):
        with fail_counts(ctx, b):
            assert ctx._fail_counts_attached is b
        assert ctx._fail_counts_attached is a
    assert ctx._fail_counts_attached is None
