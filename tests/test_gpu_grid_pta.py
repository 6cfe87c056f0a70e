"""Grid conditionals (a4, a6, a7) and the PTA CURN engine vs the reference's
golden vectors (needs an MI355X).

Grid draws are integer outcomes: indices and the written log10 rho must match
the reference EXACTLY on identical inputs (the kernels reproduce numpy's
operation order).  The PTA sweep fed the reference's rotated normals must
reproduce its chain (grid values, exact) and b (1e-9 norm-wise)."""
import numpy as np
import pytest

from oracle import gibbs_oracle as O
from tests.conftest import golden
from tests.parity_data import exact_mean_draw, normwise_rel, pta_blocks, pta_last_draw, pta_replay

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def ctx():
    from pulsar_timing_gibbsspec_amd import _lib
    return _lib.Context(0, seed=99)


def dev(a, dtype=torch.float64):
    return torch.as_tensor(np.ascontiguousarray(a), dtype=dtype).cuda()


class Keep:
    """Device copies that stay alive until the test ends.  `_lib.ptr(dev(a))` inline
    would free the temporary as soon as ptr() returns and torch's caching allocator
    would hand the same block to the next argument (aliased inputs)."""

    def __init__(self):
        self.held = []

    def __call__(self, a, dtype=torch.float64):
        from pulsar_timing_gibbsspec_amd import _lib
        if a is None:
            return None
        t = dev(a, dtype)
        self.held.append(t)
        return _lib.ptr(t)


def test_gumbel_kernel_exact(ctx):
    from pulsar_timing_gibbsspec_amd import _lib
    from pulsar_timing_gibbsspec_amd.engine import grid3
    g = golden("gumbel_j1713.npz")
    nc = g["b"].shape[0]
    tau = np.stack([O.tau_half(g["b"][c], g["gwid"]) for c in range(nc)])     # (nc, n_f)
    n_f = tau.shape[1]
    x = torch.zeros(nc, n_f, dtype=torch.float64, device="cuda")
    idx = torch.zeros(n_f * nc, dtype=torch.int32, device="cuda")
    G = grid3(float(g["rhomin"]), float(g["rhomax"]))
    K = Keep()
    _lib.check(ctx.lib.gs_rho_gumbel(ctx.handle, nc, n_f, K(tau.T), K(g["irn"].T), 1000, _lib.ptr(G),
                                     K(g["gumbel_u"]), 0, 0, _lib.ptr(x), n_f,
                                     K(np.arange(n_f, dtype=np.int32), torch.int32), _lib.ptr(idx)),
               "gs_rho_gumbel")
    want = np.stack([g["xnew"][c][g["gwind"]] for c in range(nc)])
    assert np.array_equal(x.cpu().numpy(), want)


@pytest.mark.parametrize("grid_exact", [1, 0, 2])
@pytest.mark.parametrize("kind", ["curn", "curn_red"])
def test_grid_cdf_kernels_exact(ctx, kind, grid_exact, request):
    """a6 (and a7) on every sweep's recorded inputs: indices equal to the reference's.
    grid_exact=1: numpy's operation order (bit-identical pdfs/cdfs); grid_exact=2: log-space CURN
    product and rcp-Newton ratios (pdfs within ~1e-15 relative: an index could differ only for u
    within that of a cdf value — none on the fixtures); grid_exact=0 (the default): as 2 with the
    red grid in certified f32 (rows the certificate cannot prove redone in f64)."""
    from pulsar_timing_gibbsspec_amd import _lib
    _lib.check(ctx.lib.gs_ctx_set_option(ctx.handle, _lib.OPT_GRID_EXACT, grid_exact), "set_option")
    request.addfinalizer(lambda: ctx.lib.gs_ctx_set_option(ctx.handle, _lib.OPT_GRID_EXACT, 0))
    from pulsar_timing_gibbsspec_amd.engine import grid3
    g = golden(f"pta_{kind}.npz")
    *_, rec = pta_replay(g, kind)
    P, n_f = rec[0]["tau"].shape
    Gg = grid3(float(g["rhomin_gw"]), float(g["rhomax_gw"]))
    Gr = grid3(float(g["rhomin_red"]), float(g["rhomax_red"]))
    n_param = g["x0"].size
    K = Keep()
    for ii, r in enumerate(rec):
        if kind == "curn_red":
            x = dev(g["chain"][ii][None])
            idx = torch.zeros(P * n_f, dtype=torch.int32, device="cuda")
            _lib.check(ctx.lib.gs_rho_red(ctx.handle, P, 1, n_f, K(r["tau_red"][:, :, None]),
                                          K(r["gwphi"][:, None]), 1000, _lib.ptr(Gr), K(r["u_red"][None]),
                                          0, 0, _lib.ptr(x), n_param, K(g["hind"].astype(np.int32), torch.int32),
                                          _lib.ptr(idx)), "gs_rho_red")
            got = idx.cpu().numpy()
            # the oracle keeps searchsorted-1 = -1; the device stores the wrapped index
            bad = np.nonzero(got != r["idx_red"].ravel() % 1000)[0]
            if bad.size:
                info = []
                rho = O.rho_grid(float(g["rhomin_red"]), float(g["rhomax_red"]))
                for q in bad[:5]:
                    p_, k_ = divmod(int(q), n_f)
                    ratio = r["tau_red"][p_, k_] / (r["gwphi"][k_] + rho)
                    cdf = np.cumsum(ratio * np.exp(-ratio / 2) * np.log(10))
                    cdf /= cdf.max()
                    u = r["u_red"][p_, k_]
                    info.append((p_, k_, int(got[q]), int(r["idx_red"].ravel()[q]), u,
                                 cdf[max(0, got[q] - 1):got[q] + 2].tolist(), r["tau_red"][p_, k_]))
                pytest.fail(f"sweep {ii}: {bad.size}/{got.size} red indices differ: {info}")
            assert np.array_equal(x.cpu().numpy()[0], r["x_red"]), ii
        x = dev((r["x_red"] if kind == "curn_red" else g["chain"][ii])[None])
        idx = torch.zeros(n_f, dtype=torch.int32, device="cuda")
        irn = r["irn"][:, :, None] if kind == "curn_red" else None
        _lib.check(ctx.lib.gs_rho_curn(ctx.handle, P, 1, n_f, K(r["tau"][:, :, None]), K(irn), 1000,
                                       _lib.ptr(Gg), K(r["u_curn"][None]), 0, 0, _lib.ptr(x), n_param,
                                       K(g["rind"].astype(np.int32), torch.int32), _lib.ptr(idx)),
                   "gs_rho_curn")
        assert np.array_equal(idx.cpu().numpy(), r["idx_curn"] % 1000), ii
        assert np.array_equal(x.cpu().numpy()[0], r["x_curn"]), ii


@pytest.mark.parametrize("kind,mode", [("curn", "exact"), ("curn", "sum"), ("curn_red", "exact")])
def test_pta_engine_matches_reference_chain(ctx, kind, mode):
    """PTAChains (45 pulsars) fed the reference's rotated normals and uniforms.  mode 'sum' is
    the production CURN path (PTABlockGibbs' curn_mode='auto' without per-pulsar red noise, the
    benched line and the one a pulsar-sharded run all-reduces for): gs_tau_sum_fx_b ->
    gs_fx_to_double -> gs_rho_curn_sum must pick the reference's grid index on every sweep, so
    the recorded x chain equals the reference's exactly and the gate matches each sweep."""
    from pulsar_timing_gibbsspec_amd.engine import DeviceModel, PTAChains
    from pulsar_timing_gibbsspec_amd import synthetic
    g = golden(f"pta_{kind}.npz")
    chain, bhist, bfin, _, _, rec = pta_replay(g, kind, rotate=True)
    pta = synthetic.array_pta(kind=kind, seed=0)
    T, N, R = pta.get_basis(), pta.get_ndiag({}), pta.get_residuals()
    gwid = [np.asarray(x) for x in g["gwid"]]
    fixed = [np.full(T[p].shape[1] - 60, 1e-40) for p in range(len(T))]
    model = DeviceModel(ctx, T, N, R, gwid, fixed)
    for p in (0, 17, 44):                                  # same TNT/d as the fixture's
        a, b = model.tnt_host(p)
        m = a.shape[0]
        o = int(np.sum(g["m"][:p] ** 2))
        assert normwise_rel(a, g["TNT"][o:o + m * m].reshape(m, m)) < 1e-12
    hind = g["hind"]
    red_col = hind.reshape(len(T), -1) if kind == "curn_red" else None
    eng = PTAChains(model, g["x0"].size, g["rind"], red_col, (float(g["rhomin_gw"]), float(g["rhomax_gw"])),
                    (float(g["rhomin_red"]), float(g["rhomax_red"])), 1, g["x0"], curn_mode=mode)
    xr = torch.zeros(len(rec), 1, g["x0"].size, dtype=torch.float64, device="cuda")
    for ii, r in enumerate(rec):
        eng.sweep(x_rec=xr[ii], z0=dev(r["z0"]) if ii == 0 else None,
                  z=dev(r["z"]) if r["gate"] else None,
                  u_red=dev(r["u_red"][None]) if kind == "curn_red" else None,
                  u_curn=dev(r["u_curn"][None]))
        assert bool(eng.gate.cpu()[0]) == r["gate"], ii
    assert np.array_equal(xr.cpu().numpy()[:, 0], g["chain"])
    eng.check_fx()
    b = eng.b.cpu().numpy()
    # final b per pulsar vs the reference draw with an exact mean (1e-9); the
    # reference's own fp64 SVD mean is off by up to ~3e-8 on these systems
    # (tests/test_oracle_golden.py::test_reference_svd_mean_error), so the raw
    # comparison is bounded by that error + 1e-9.
    TNTs, ds = pta_blocks(g)
    x, zl = pta_last_draw(g, kind, rec)
    off = np.concatenate([[0], np.cumsum(g["m"])])
    n_f = len(g["rind"])
    for p in range(len(T)):
        phi_f = 10 ** (2 * x[g["rind"]])
        if kind == "curn_red":
            phi_f = phi_f + 10 ** (2 * x[g["hind"][p * n_f:(p + 1) * n_f]])
        ph = np.full(g["m"][p], 1e-40)
        ph[gwid[p]] = 1.0 / np.repeat(phi_f, 2)
        bx = exact_mean_draw(TNTs[p], ds[p], ph, zl[p])
        bp = b[p, :g["m"][p]]
        assert normwise_rel(bp, bx) < 1e-9, p
        bref = g["b_final"][off[p]:off[p + 1]]
        assert normwise_rel(bp, bref) <= normwise_rel(bref, bx) + 1e-9, p
    assert not eng.info.cpu().numpy().any()


def test_pta_block_gibbs_surface(tmp_path):
    from pulsar_timing_gibbsspec_amd import PTABlockGibbs, synthetic
    pta = synthetic.array_pta(kind="curn_red", n_psr=6, seed=3)
    gb = PTABlockGibbs(pta, hypersample="conditional", redsample="conditional", nchains=8, seed=1)
    x0 = np.concatenate([p.sample().flatten() for p in gb.params])
    chain = gb.sample(x0, outdir=str(tmp_path), niter=120)
    assert chain.shape == (120, 6 * 30 + 30)
    saved = np.loadtxt(tmp_path / "chain.txt")
    assert saved.shape == (101, 210)
    assert np.array_equal(saved, chain[:101])
    assert np.load(tmp_path / "chains.npy").shape == (8, 101, 210)
    gw = chain[1:, gb.get_rho_param_indices()]
    assert np.all(gw >= -9.0) and np.all(gw <= -4.0)
    red = chain[1:, gb.get_hyper_param_indices()]
    assert np.all(red >= -10.0) and np.all(red <= -4.0)
    b = gb.update_b(chain[-1])
    assert len(b) == 6 and all(np.all(np.isfinite(bb)) for bb in b)


def test_pta_resume(tmp_path):
    """PTABlockGibbs resume (pta_gibbs.py:642-661): with the device state saved next to
    chain.txt the resumed run equals the uninterrupted one bit for bit (every chain); from
    chain.txt alone (the reference's own files) b is redrawn from the last row first, so the
    resumed rows stay finite and inside the prior instead of the reference's b = 0 ->
    tau = 0 -> 0/0 CDF -> every common rho pinned to the top grid point."""
    import os
    from pulsar_timing_gibbsspec_amd import PTABlockGibbs, synthetic
    pta = synthetic.array_pta(kind="curn_red", n_psr=5, seed=3)

    def new():
        return PTABlockGibbs(pta, hypersample="conditional", redsample="conditional", nchains=4, seed=9)
    x0 = np.concatenate([p.sample().flatten() for p in new().params])
    full = new()
    full.sample(x0, outdir=str(tmp_path / "a"), niter=230)
    part = new()
    part.sample(x0, outdir=str(tmp_path / "b"), niter=150)            # saves rows [:101] + state
    res = new()
    chain = res.sample(x0, outdir=str(tmp_path / "b"), niter=230, resume=True)
    assert np.array_equal(chain, full.chain)
    assert np.array_equal(res.chains, full.chains)
    os.remove(tmp_path / "b" / "gibbs_state.npz")
    np.savetxt(tmp_path / "b" / "chain.txt", full.chain[:101])
    cold = new()
    c2 = cold.sample(x0, outdir=str(tmp_path / "b"), niter=160, resume=True)
    assert np.array_equal(c2[101], c2[100])                            # the reference's repeated row
    gw = c2[102:, cold.get_rho_param_indices()]
    assert np.all(np.isfinite(gw)) and gw.min() >= -9.0 and gw.max() <= -4.0
    assert not np.all(gw == gw.max())                                  # not pinned to rho_max


@pytest.mark.parametrize("kind,nsh", [("curn", 2), ("curn_red", 2), ("curn_plred", 2), ("curn_plred", 3)])
def test_pulsar_sharded_engine_bit_identical(kind, nsh):
    """nsh pulsar shards (own context, own DeviceModel) exchanging [tau | x_red] slabs
    reproduce the unsharded engine's chains bit for bit under device Philox
    (global chain and pulsar ids in the counters).  curn_plred: the red MH block of the
    reference's default redsample='mh' runs pulsar-sharded -- each shard applies the steps of its
    own pulsars from the common step table, the power-law (log10_A, gamma) travel in the slab."""
    from pulsar_timing_gibbsspec_amd import _lib, synthetic
    from pulsar_timing_gibbsspec_amd.distributed import shard_range
    from pulsar_timing_gibbsspec_amd.engine import DeviceModel, PTAChains
    from pulsar_timing_gibbsspec_amd.pta_hyper import HyperSpec
    pta = synthetic.array_pta(kind=kind, n_psr=9, seed=2)
    T, N, R = pta.get_basis(), pta.get_ndiag({}), pta.get_residuals()
    names = pta.param_names
    rind = [i for i, n in enumerate(names) if "rho" in n and "gw" in n]
    hind = np.array([i for i, n in enumerate(names) if "red" in n and "rho" in n])
    red_col = hind.reshape(len(T), -1) if kind == "curn_red" else None
    gwid = [np.arange(t.shape[1] - 60, t.shape[1]) for t in T]
    fixed = [np.full(t.shape[1] - 60, 1e-40) for t in T]
    C, S = 16, 6
    rng = np.random.default_rng(0)
    x0 = rng.uniform(-9, -4, (C, len(names)))
    bounds = ((1e-18, 1e-8), (1e-20, 1e-8))
    hy = {}
    if kind == "curn_plred":
        hidx = np.array([i for i, n in enumerate(names) if "red" in n and ("log10_A" in n or "gamma" in n)])
        sigs = [s for s in (pta.signals[k] for k in pta.signals) if "red" in s.name]
        spec = HyperSpec(pta, pta.params, sigs, hidx, np.zeros(len(names)), 30, "cuda")
        x0[:, spec.hind] = rng.uniform(spec.hlo_host, spec.hhi_host, (C, spec.n_h))
        hy = dict(hyper=spec, hyper_acl=9, hyper_warmup=30)

    ref_ctx = _lib.Context(0, seed=77)
    ref = PTAChains(DeviceModel(ref_ctx, T, N, R, gwid, fixed), len(names), rind, red_col, *bounds, C, x0, **hy)
    xr_ref = torch.zeros(S, C, len(names), dtype=torch.float64, device="cuda")
    for i in range(S):
        ref.sweep(x_rec=xr_ref[i])

    shards = []
    for r in range(nsh):
        lo, hi = shard_range(len(T), r, nsh)
        ctx = _lib.Context(0, seed=77)
        mdl = DeviceModel(ctx, T[lo:hi], N[lo:hi], R[lo:hi], gwid[lo:hi], fixed[lo:hi])
        shards.append(PTAChains(mdl, len(names), rind, red_col, *bounds, C, x0, P_global=len(T), psr_lo=lo,
                                gather=lambda s: s, **hy))
    xr = [torch.zeros(S, C, len(names), dtype=torch.float64, device="cuda") for _ in range(nsh)]
    for i in range(S):
        slabs = [sh.sweep_begin(x_rec=xr[j][i]) for j, sh in enumerate(shards)]
        glob = torch.cat(slabs, dim=0)            # the all-gather, in global pulsar order
        for sh in shards:
            sh.sweep_end(glob)
    for j in range(nsh):
        assert torch.equal(xr[j], xr_ref), j
    if kind == "curn_plred":
        assert not torch.equal(xr_ref[-1][:, spec.hind], xr_ref[0][:, spec.hind])     # the block moved
        acc = sum(sh.hyper.acc_total for sh in shards)
        assert torch.equal(acc, ref.hyper.acc_total)
    bref = ref.b.view(len(T), C, -1)
    for r, sh in enumerate(shards):
        lo, hi = shard_range(len(T), r, nsh)
        bs = sh.b.view(hi - lo, C, -1)
        w = bs.shape[2]
        assert torch.equal(bs, bref[lo:hi, :, :w]) and not bref[lo:hi, :, w:].any()


def test_one_rank_gather_warmup_without_process_group():
    """A pulsar-sharded engine whose exchange is a 1-rank gather (gather=lambda s: s: one shard holding
    every pulsar, no torch.distributed process group) runs the red block's sweep-0 warm-up with
    aclength_hyper left to it (hyper_acl=None): distributed.allreduce_sum passes the local records
    through, and the chains, aclength_hyper and acceptance equal the unsharded engine's."""
    import torch.distributed as dist
    from pulsar_timing_gibbsspec_amd import _lib, synthetic
    from pulsar_timing_gibbsspec_amd.engine import DeviceModel, PTAChains
    from pulsar_timing_gibbsspec_amd.pta_hyper import HyperSpec
    assert not dist.is_initialized()
    pta = synthetic.array_pta(kind="curn_plred", n_psr=5, seed=2)
    T, N, R = pta.get_basis(), pta.get_ndiag({}), pta.get_residuals()
    names = pta.param_names
    rind = [i for i, n in enumerate(names) if "rho" in n and "gw" in n]
    gwid = [np.arange(t.shape[1] - 60, t.shape[1]) for t in T]
    fixed = [np.full(t.shape[1] - 60, 1e-40) for t in T]
    hidx = np.array([i for i, n in enumerate(names) if "red" in n and ("log10_A" in n or "gamma" in n)])
    sigs = [s for s in (pta.signals[k] for k in pta.signals) if "red" in s.name]
    C, S = 16, 4
    rng = np.random.default_rng(0)
    x0 = rng.uniform(-9, -4, (C, len(names)))
    engs, recs = [], []
    for sharded in (False, True):
        spec = HyperSpec(pta, pta.params, sigs, hidx, np.zeros(len(names)), 30, "cuda")
        if not sharded:
            x0[:, spec.hind] = rng.uniform(spec.hlo_host, spec.hhi_host, (C, spec.n_h))
        ex = dict(P_global=len(T), psr_lo=0, gather=lambda s: s) if sharded else {}
        eng = PTAChains(DeviceModel(_lib.Context(0, seed=91), T, N, R, gwid, fixed), len(names), rind, None,
                        (1e-18, 1e-8), (1e-20, 1e-8), C, x0, hyper=spec, hyper_warmup=30, **ex)
        assert eng.sharded == sharded
        xr = torch.zeros(S, C, len(names), dtype=torch.float64, device="cuda")
        for i in range(S):
            if sharded:
                eng.sweep_end(eng.sweep_begin(x_rec=xr[i]))
            else:
                eng.sweep(x_rec=xr[i])
        engs.append(eng)
        recs.append(xr)
    assert torch.equal(recs[0], recs[1])
    assert engs[0].hyper_acl == engs[1].hyper_acl and engs[0].hyper_acl >= 1
    assert np.array_equal(engs[0].hyper_acceptance(), engs[1].hyper_acceptance())


def test_curn_sum_kernel_matches_reference(ctx):
    """gs_tau_sum + gs_rho_curn_sum (the sufficient-statistic CURN draw a sharded run
    all-reduces for) pick the reference's grid index on every sweep of the fixture."""
    from pulsar_timing_gibbsspec_amd import _lib
    from pulsar_timing_gibbsspec_amd.engine import grid3
    g = golden("pta_curn.npz")
    *_, rec = pta_replay(g, "curn")
    P, n_f = rec[0]["tau"].shape
    Gg = grid3(float(g["rhomin_gw"]), float(g["rhomax_gw"]))
    n_param = g["x0"].size
    K = Keep()
    for ii, r in enumerate(rec):
        S = torch.zeros(n_f, 1, dtype=torch.float64, device="cuda")
        _lib.check(ctx.lib.gs_tau_sum(ctx.handle, P, 1, n_f, K(r["tau"][:, :, None]), _lib.ptr(S)), "gs_tau_sum")
        assert np.allclose(S.cpu().numpy()[:, 0], r["tau"].sum(axis=0), rtol=1e-15, atol=0)
        x = dev(g["chain"][ii][None])
        idx = torch.zeros(n_f, dtype=torch.int32, device="cuda")
        _lib.check(ctx.lib.gs_rho_curn_sum(ctx.handle, P, 1, n_f, _lib.ptr(S), 1000, _lib.ptr(Gg),
                                           K(r["u_curn"][None]), 0, 0, _lib.ptr(x), n_param,
                                           K(g["rind"].astype(np.int32), torch.int32), _lib.ptr(idx)),
                   "gs_rho_curn_sum")
        assert np.array_equal(idx.cpu().numpy(), r["idx_curn"] % 1000), ii
        assert np.array_equal(x.cpu().numpy()[0], r["x_curn"]), ii


def test_curn_sum_fixed_point_matches_reference(ctx):
    """The production CURN kernels open loop on every fixture sweep's recorded tau: the exact
    fixed-point digits (gs_tau_sum_fx, the quantity a pulsar-sharded run all-reduces) ->
    gs_fx_to_double -> gs_rho_curn_sum give the reference's grid index (pta_gibbs.py:181-214)
    and the sums equal the exactly rounded sum of the tau (math.fsum) to 1 ulp; the in-kernel
    variant from b (gs_tau_sum_fx_b) gives the same digits as tau -> gs_tau_sum_fx."""
    import math
    from pulsar_timing_gibbsspec_amd import _lib
    from pulsar_timing_gibbsspec_amd.engine import grid3
    g = golden("pta_curn.npz")
    _, bhist, _, _, _, rec = pta_replay(g, "curn")
    P, n_f = rec[0]["tau"].shape
    Gg = grid3(float(g["rhomin_gw"]), float(g["rhomax_gw"]))
    e0 = int(np.floor(np.log2(float(g["rhomin_gw"])))) - 64
    n_param = g["x0"].size
    K = Keep()
    ovf = torch.zeros(1, dtype=torch.int32, device="cuda")
    for ii, r in enumerate(rec):
        acc = torch.zeros(3, n_f, 1, dtype=torch.int64, device="cuda")
        _lib.check(ctx.lib.gs_tau_sum_fx(ctx.handle, P, 1, n_f, K(r["tau"][:, :, None]), e0, _lib.ptr(acc),
                                         _lib.ptr(ovf)), "gs_tau_sum_fx")
        S = torch.zeros(n_f, 1, dtype=torch.float64, device="cuda")
        _lib.check(ctx.lib.gs_fx_to_double(ctx.handle, n_f, e0, _lib.ptr(acc), _lib.ptr(S)), "gs_fx_to_double")
        Sh = S.cpu().numpy()[:, 0]
        want = np.array([math.fsum(r["tau"][:, k]) for k in range(n_f)])
        assert np.all(np.abs(Sh - want) <= np.spacing(want)), ii
        x = dev(g["chain"][ii][None])
        idx = torch.zeros(n_f, dtype=torch.int32, device="cuda")
        _lib.check(ctx.lib.gs_rho_curn_sum(ctx.handle, P, 1, n_f, _lib.ptr(S), 1000, _lib.ptr(Gg),
                                           K(r["u_curn"][None]), 0, 0, _lib.ptr(x), n_param,
                                           K(g["rind"].astype(np.int32), torch.int32), _lib.ptr(idx)),
                   "gs_rho_curn_sum")
        assert np.array_equal(idx.cpu().numpy(), r["idx_curn"] % 1000), ii
        assert np.array_equal(x.cpu().numpy()[0], r["x_curn"]), ii
    assert int(ovf.item()) == 0
    # gs_tau_sum_fx_b straight from b (the engine's fused pass) == tau -> gs_tau_sum_fx
    m = g["m"]
    ldb = int(m.max())
    off = np.concatenate([[0], np.cumsum(m)])
    fidx = np.stack([np.asarray(gw, np.int32) for gw in g["gwid"]])
    for ii in (1, len(rec) - 1):
        bb = np.zeros((P, ldb))
        for p in range(P):
            bb[p, :m[p]] = bhist[ii][off[p]:off[p + 1]]
        tau = np.stack([O.tau_full(bb[p, :m[p]], g["gwid"][p]) for p in range(P)])
        a1 = torch.zeros(3, n_f, 1, dtype=torch.int64, device="cuda")
        a2 = torch.zeros_like(a1)
        _lib.check(ctx.lib.gs_tau_sum_fx(ctx.handle, P, 1, n_f, K(tau[:, :, None]), e0, _lib.ptr(a1), None),
                   "gs_tau_sum_fx")
        _lib.check(ctx.lib.gs_tau_sum_fx_b(ctx.handle, P, 1, 2 * n_f, ldb, K(fidx, torch.int32), K(bb), e0,
                                           _lib.ptr(a2), None), "gs_tau_sum_fx_b")
        assert torch.equal(a1, a2), ii


def test_curn_sum_overflow_raises(ctx):
    """A tau outside the fixed-point window (here b = 1e30) must not feed a silently truncated S
    into the CURN draw: PTAChains.check_fx raises."""
    from pulsar_timing_gibbsspec_amd import synthetic
    from pulsar_timing_gibbsspec_amd.engine import DeviceModel, PTAChains
    pta = synthetic.array_pta(kind="curn", n_psr=3, seed=2)
    T, N, R = pta.get_basis(), pta.get_ndiag({}), pta.get_residuals()
    names = pta.param_names
    rind = [i for i, n in enumerate(names) if "rho" in n and "gw" in n]
    gwid = [np.arange(t.shape[1] - 60, t.shape[1]) for t in T]
    fixed = [np.full(t.shape[1] - 60, 1e-40) for t in T]
    x0 = np.random.default_rng(0).uniform(-9, -4, (4, len(names)))
    eng = PTAChains(DeviceModel(ctx, T, N, R, gwid, fixed), len(names), rind, None, (1e-18, 1e-8), (1e-18, 1e-8),
                    4, x0, curn_mode="sum")
    eng.sweep()
    eng.check_fx()
    eng.b.fill_(1e30)
    eng.sweep()
    with pytest.raises(RuntimeError, match="fixed-point window"):
        eng.check_fx()


def test_curn_sum_sharded_engine_matches_unsharded():
    """curn_mode='sum': two pulsar shards exchanging partial tau sums (the all-reduce)
    reproduce the unsharded sum-mode chains under device Philox; the unsharded
    sum-mode chain itself stays within the exact engine's posterior (same grid)."""
    from pulsar_timing_gibbsspec_amd import _lib, synthetic
    from pulsar_timing_gibbsspec_amd.distributed import shard_range
    from pulsar_timing_gibbsspec_amd.engine import DeviceModel, PTAChains
    pta = synthetic.array_pta(kind="curn", n_psr=9, seed=2)
    T, N, R = pta.get_basis(), pta.get_ndiag({}), pta.get_residuals()
    names = pta.param_names
    rind = [i for i, n in enumerate(names) if "rho" in n and "gw" in n]
    gwid = [np.arange(t.shape[1] - 60, t.shape[1]) for t in T]
    fixed = [np.full(t.shape[1] - 60, 1e-40) for t in T]
    C, S = 16, 6
    x0 = np.random.default_rng(0).uniform(-9, -4, (C, len(names)))
    bounds = ((1e-18, 1e-8), (1e-20, 1e-8))
    ref = PTAChains(DeviceModel(_lib.Context(0, seed=78), T, N, R, gwid, fixed), len(names), rind, None,
                    *bounds, C, x0, curn_mode="sum")
    xr_ref = torch.zeros(S, C, len(names), dtype=torch.float64, device="cuda")
    for i in range(S):
        ref.sweep(x_rec=xr_ref[i])
    shards = []
    for r in range(2):
        lo, hi = shard_range(len(T), r, 2)
        mdl = DeviceModel(_lib.Context(0, seed=78), T[lo:hi], N[lo:hi], R[lo:hi], gwid[lo:hi], fixed[lo:hi])
        shards.append(PTAChains(mdl, len(names), rind, None, *bounds, C, x0, P_global=len(T), psr_lo=lo,
                                curn_mode="sum", allreduce=lambda s: s))
    xr = [torch.zeros(S, C, len(names), dtype=torch.float64, device="cuda") for _ in range(2)]
    for i in range(S):
        parts = [sh.sweep_begin(x_rec=xr[j][i]) for j, sh in enumerate(shards)]
        tot = parts[0] + parts[1]                     # the all-reduce
        for sh in shards:
            sh.sweep_end(tot.clone())
    assert torch.equal(xr[0], xr[1])
    assert torch.equal(xr[0], xr_ref)
    gw = xr_ref[:, :, rind].cpu().numpy()
    assert np.isfinite(gw).all() and (gw >= -9).all() and (gw <= -4).all()


@pytest.mark.parametrize("kind,mode", [("curn", "sum"), ("curn_red", "exact"), ("curn_plred", "exact")])
def test_graph_replay_equals_eager_sweeps(kind, mode):
    """hipGraph-captured sweeps (device sweep counter advanced inside the graph) replay
    to the same chains as eager sweeps, replay after replay.  curn_plred (redsample='mh'): the red
    MH block inside the graph too, and its acceptance counts (a device add replayed with the graph,
    the step count kept on the host per replay) equal the eager engine's."""
    from pulsar_timing_gibbsspec_amd import _lib, synthetic
    from pulsar_timing_gibbsspec_amd.engine import DeviceModel, PTAChains
    pta = synthetic.array_pta(kind=kind, n_psr=7, seed=4)
    T, N, R = pta.get_basis(), pta.get_ndiag({}), pta.get_residuals()
    names = pta.param_names
    rind = [i for i, n in enumerate(names) if "rho" in n and "gw" in n]
    hind = np.array([i for i, n in enumerate(names) if "red" in n and "rho" in n])
    red_col = hind.reshape(len(T), -1) if kind == "curn_red" else None
    gwid = [np.arange(t.shape[1] - 60, t.shape[1]) for t in T]
    fixed = [np.full(t.shape[1] - 60, 1e-40) for t in T]
    C, K = 8, 4
    rng = np.random.default_rng(1)
    x0 = rng.uniform(-9, -4, (C, len(names)))
    bounds = ((1e-18, 1e-8), (1e-20, 1e-8))
    hy = {}
    if kind == "curn_plred":
        from pulsar_timing_gibbsspec_amd.pta_hyper import HyperSpec
        hidx = np.array([i for i, n in enumerate(names) if "red" in n and ("log10_A" in n or "gamma" in n)])
        sigs = [s for s in (pta.signals[k] for k in pta.signals) if "red" in s.name]
        spec = HyperSpec(pta, pta.params, sigs, hidx, np.zeros(len(names)), 30, "cuda")
        x0[:, spec.hind] = rng.uniform(spec.hlo_host, spec.hhi_host, (C, spec.n_h))
        hy = dict(hyper=spec, hyper_acl=7, hyper_warmup=25)

    def engine():
        ctx = _lib.Context(0, seed=5)
        return PTAChains(DeviceModel(ctx, T, N, R, gwid, fixed), len(names), rind, red_col, *bounds, C, x0,
                         curn_mode=mode, **hy)
    ref = engine()
    xr = torch.zeros(1 + 3 * K, C, len(names), dtype=torch.float64, device="cuda")
    for i in range(1 + 3 * K):
        ref.sweep(x_rec=xr[i])
    g = engine()
    xg = torch.zeros_like(xr)
    g.sweep(x_rec=xg[0])
    g.capture(K)
    for r in range(3):
        g.replay()
        xg[1 + r * K:1 + (r + 1) * K].copy_(g.graph_rec)
    torch.cuda.synchronize()
    assert torch.equal(xg, xr)
    if kind == "curn_plred":
        assert g.hyper.steps_total == ref.hyper.steps_total == 25 + 3 * K * 7
        assert torch.equal(g.hyper.acc_total, ref.hyper.acc_total)
        assert np.array_equal(g.hyper_acceptance(), ref.hyper_acceptance())


def test_tau_sum_fixed_point_kernels():
    """gs_tau_sum_fx: the int64 digits equal the Python-integer restatement bit for bit
    (tests/test_distributed.fx_digits); gs_fx_to_double: the double those digits stand for,
    correctly rounded (or at most 1 ulp off), identical for digits summed over any sharding."""
    import torch
    from pulsar_timing_gibbsspec_amd import _lib
    from pulsar_timing_gibbsspec_amd._lib import check, ptr
    from tests.test_distributed import _tau_case, fx_digits, fx_value
    tau, e0 = _tau_case()
    P, n_f, C = tau.shape
    ctx = _lib.Context(0, seed=1)
    t = torch.as_tensor(tau, device="cuda")
    acc = torch.zeros(3, n_f, C, dtype=torch.int64, device="cuda")
    ovf = torch.zeros(1, dtype=torch.int32, device="cuda")
    check(ctx.lib.gs_tau_sum_fx(ctx.handle, P, C, n_f, ptr(t), e0, ptr(acc), ptr(ovf)), "gs_tau_sum_fx")
    want = fx_digits(tau, e0)
    assert np.array_equal(acc.cpu().numpy(), want) and int(ovf) == 0
    # shard digits (3 uneven blocks) added as int64 -> the same digits
    parts = torch.zeros_like(acc)
    for lo, hi in ((0, 7), (7, 30), (30, P)):
        a = torch.zeros_like(acc)
        check(ctx.lib.gs_tau_sum_fx(ctx.handle, hi - lo, C, n_f, ptr(t[lo:hi].contiguous()), e0, ptr(a), None), "fx")
        parts += a
    assert torch.equal(parts, acc)
    S = torch.empty(n_f, C, dtype=torch.float64, device="cuda")
    check(ctx.lib.gs_fx_to_double(ctx.handle, n_f * C, e0, ptr(acc), ptr(S)), "gs_fx_to_double")
    got, ref = S.cpu().numpy().ravel(), fx_value(want, e0)
    assert np.all(np.abs(got - ref) <= np.spacing(ref))
    # overflow / invalid input is flagged
    t[0, 0, 0] = -1.0
    check(ctx.lib.gs_tau_sum_fx(ctx.handle, P, C, n_f, ptr(t), e0, ptr(acc), ptr(ovf)), "gs_tau_sum_fx")
    assert int(ovf) == 1


def test_red_grid_certified_f32_matches_exact(ctx, request):
    """The default red-grid draw (GS_OPT_GRID_EXACT = 0: f32 points + per-row error certificate,
    f64 redo of unproven rows) on 86k random rows spanning 16 decades of tau and 10 of gw: the
    same index as the f64 wave kernel (= 2) on every row, and as numpy's operation order (= 1) on
    every row whose u is not placed on a cdf value.  Rows with u exactly on a cdf value (computed
    in f64 as the reference does) cannot be certified in f32: they take the f64 path (counted)."""
    from pulsar_timing_gibbsspec_amd import _lib
    from pulsar_timing_gibbsspec_amd.engine import grid3
    request.addfinalizer(lambda: ctx.lib.gs_ctx_set_option(ctx.handle, _lib.OPT_GRID_EXACT, 0))
    rng = np.random.default_rng(11)
    P, n_f, C = 45, 30, 64
    lo, hi = 1e-20, 1e-8
    tau = 10 ** rng.uniform(-22, -6, (P, n_f, C))
    gw = 10 ** rng.uniform(-18, -8, (n_f, C))
    u = rng.random((C, P, n_f))
    # adversarial rows: u exactly at the f64 cdf value of a random index
    rho = O.rho_grid(lo, hi)
    adv = [(p, k, c) for p, k, c in zip(rng.integers(0, P, 40), rng.integers(0, n_f, 40), rng.integers(0, C, 40))]
    for p, k, c in adv:
        ratio = tau[p, k, c] / (gw[k, c] + rho)
        cdf = np.cumsum(ratio * np.exp(-ratio / 2) * np.log(10))
        cdf /= cdf.max()
        j = int(rng.integers(100, 900))
        u[c, p, k] = cdf[j]
    G = grid3(lo, hi)
    xcol = torch.arange(P * n_f, dtype=torch.int32, device="cuda")
    out, nfbs = {}, {}
    fb = torch.zeros(1, dtype=torch.int32, device="cuda")
    for mode in (1, 2, 3, 0):
        _lib.check(ctx.lib.gs_ctx_set_option(ctx.handle, _lib.OPT_GRID_EXACT, mode), "set_option")
        x = torch.zeros(C, P * n_f, dtype=torch.float64, device="cuda")
        idx = torch.zeros(P * n_f * C, dtype=torch.int32, device="cuda")
        K = Keep()
        _lib.check(ctx.lib.gs_ctx_set_grid_fallback_counter(ctx.handle, _lib.ptr(fb)), "counter")
        try:
            _lib.check(ctx.lib.gs_rho_red(ctx.handle, P, C, n_f, K(tau), K(gw), 1000, _lib.ptr(G), K(u), 0, 0,
                                          _lib.ptr(x), P * n_f, _lib.ptr(xcol), _lib.ptr(idx)), "gs_rho_red")
        finally:
            _lib.check(ctx.lib.gs_ctx_set_grid_fallback_counter(ctx.handle, None), "counter")
        out[mode] = idx.cpu().numpy()
        nfbs[mode] = int(fb)
        fb.zero_()
    nfb = nfbs[0]
    advset = {(p * n_f + k) * C + c for p, k, c in adv}   # row r = (p * n_f + k) * C + c
    # mode 0 = 16 lanes per row (k_rho_red_cert16), 3 = the round-3 64-lane certified kernel
    assert np.array_equal(out[0], out[2]), int(np.sum(out[0] != out[2]))
    assert np.array_equal(out[3], out[2]), int(np.sum(out[3] != out[2]))
    keep = np.ones(out[0].size, bool)
    keep[list(advset)] = False
    bad = np.nonzero((out[0] != out[1]) & keep)[0]
    if bad.size:
        info = []
        for q in bad[:6]:
            p_, rem = divmod(int(q), n_f * C)
            k_, c_ = divmod(rem, C)
            ratio = tau[p_, k_, c_] / (gw[k_, c_] + rho)
            cdf = np.cumsum(ratio * np.exp(-ratio / 2) * np.log(10))
            cdf /= cdf.max()
            j0 = int(out[1][q])
            info.append(dict(row=int(q), adversarial=int(q) in advset, cert=int(out[0][q]), exact=j0,
                             u=float(u[c_, p_, k_]), cdf=cdf[max(0, j0 - 1):j0 + 2].tolist(),
                             tau=float(tau[p_, k_, c_]), gw=float(gw[k_, c_])))
        pytest.fail(f"{bad.size} rows differ (fallbacks {nfb}): {info}")
    # the adversarial rows, and ~1-2 % of the others (u within the certificate's margin of one of
    # ~1000 cdf values)
    assert len(adv) <= nfbs[3] < 0.03 * out[0].size, nfbs[3]
    assert len(adv) <= nfb < 0.03 * out[0].size, nfb


@pytest.mark.parametrize("ngrid", [1, 2, 3, 17, 63, 64, 65, 127, 128, 500, 999, 1023, 1024, 1025])
def test_red_grid_certified_grid_sizes(ctx, request, ngrid):
    """k_rho_red_cert16 (64 points per lane, 16 lanes per row) at grid sizes around its lane and
    row boundaries -- lanes with no points, one partial lane, exactly full rows -- against the f64
    kernel (GS_OPT_GRID_EXACT = 2): the same index on every row (ngrid > 1024 takes the
    lane-per-row kernel in both modes)."""
    from pulsar_timing_gibbsspec_amd import _lib
    from pulsar_timing_gibbsspec_amd.engine import grid3
    request.addfinalizer(lambda: ctx.lib.gs_ctx_set_option(ctx.handle, _lib.OPT_GRID_EXACT, 0))
    rng = np.random.default_rng(ngrid)
    P, n_f, C = 3, 5, 67            # 1005 rows: a short last wave
    tau = 10 ** rng.uniform(-22, -6, (P, n_f, C))
    gw = 10 ** rng.uniform(-18, -8, (n_f, C))
    u = rng.random((C, P, n_f))
    G = grid3(1e-20, 1e-8, n=ngrid)
    xcol = torch.arange(P * n_f, dtype=torch.int32, device="cuda")
    out = {}
    for mode in (2, 0):
        _lib.check(ctx.lib.gs_ctx_set_option(ctx.handle, _lib.OPT_GRID_EXACT, mode), "set_option")
        x = torch.zeros(C, P * n_f, dtype=torch.float64, device="cuda")
        idx = torch.full((P * n_f * C,), -7, dtype=torch.int32, device="cuda")
        K = Keep()
        _lib.check(ctx.lib.gs_rho_red(ctx.handle, P, C, n_f, K(tau), K(gw), ngrid, _lib.ptr(G), K(u), 0, 0,
                                      _lib.ptr(x), P * n_f, _lib.ptr(xcol), _lib.ptr(idx)), "gs_rho_red")
        out[mode] = (idx.cpu().numpy(), x.cpu().numpy())
    assert out[0][0].min() >= 0 and out[0][0].max() < ngrid
    assert np.array_equal(out[0][0], out[2][0]), int(np.sum(out[0][0] != out[2][0]))
    assert np.array_equal(out[0][1], out[2][1])


@pytest.mark.parametrize("with_red,P,lo", [(True, 45, 1e-18), (False, 45, 1e-18), (True, 12, 1e-18),
                                            (True, 45, 1e-34)])
def test_curn_fast_matches_numpy_order_on_random_rows(ctx, request, with_red, P, lo):
    """The default CURN draw (k_rho_curn_fast: grouped-polynomial N / D product, log-space pdf)
    against numpy's operation order (GS_OPT_GRID_EXACT = 1) on random rows of P pulsars
    whose tau follows each row's own rho (ratio / 2 ~ Exp(1) at rho_true, so the product over
    pulsars stays representable as in a real chain), with and without per-pulsar red noise
    spanning 9 decades: the same index on every row (pdfs agree to ~1e-15 relative, so a row could
    only differ if u fell that close to a cdf value).  P = 45 takes 5-pulsar coefficient groups,
    P = 12 4-pulsar groups; a grid down to rho = 1e-34 (< 1e-30) rescales after every group."""
    from pulsar_timing_gibbsspec_amd import _lib
    from pulsar_timing_gibbsspec_amd.engine import grid3
    request.addfinalizer(lambda: ctx.lib.gs_ctx_set_option(ctx.handle, _lib.OPT_GRID_EXACT, 0))
    rng = np.random.default_rng(5 + with_red + P)
    n_f, C = 30, 256
    hi = 1e-8
    rho_true = 10 ** rng.uniform(-16, -9, (1, n_f, C))
    irn = 10 ** rng.uniform(-18, -9, (P, n_f, C)) if with_red else np.zeros((P, n_f, C))
    tau = (irn + rho_true) * rng.exponential(2.0, (P, n_f, C))
    u = rng.random((C, n_f))
    G = grid3(lo, hi)
    xcol = torch.arange(n_f, dtype=torch.int32, device="cuda")
    out = {}
    for mode in (1, 0):
        _lib.check(ctx.lib.gs_ctx_set_option(ctx.handle, _lib.OPT_GRID_EXACT, mode), "set_option")
        x = torch.zeros(C, n_f, dtype=torch.float64, device="cuda")
        idx = torch.zeros(n_f * C, dtype=torch.int32, device="cuda")
        K = Keep()
        _lib.check(ctx.lib.gs_rho_curn(ctx.handle, P, C, n_f, K(tau), K(irn) if with_red else None, 1000,
                                       _lib.ptr(G), K(u), 0, 0, _lib.ptr(x), n_f, _lib.ptr(xcol), _lib.ptr(idx)),
                   "gs_rho_curn")
        out[mode] = idx.cpu().numpy()
    bad = np.nonzero(out[0] != out[1])[0]
    assert bad.size == 0, (bad.size, bad[:8].tolist(), out[0][bad[:8]].tolist(), out[1][bad[:8]].tolist())
    # the draws are spread over the grid, not piled on one end
    assert len(np.unique(out[1])) > 150


@pytest.mark.parametrize("phi_shared,masked,nf,small_nm", [(False, False, 60, False), (True, True, 60, False),
                                                           (False, True, 60, True), (True, False, 40, False)])
def test_bdraw_tiled_equals_row_major(ctx, phi_shared, masked, nf, small_nm):
    """gs_bdraw_tiled (register-tile copies of the model blocks, gs_model_tile) draws the same b,
    bit for bit, as gs_bdraw on the row-major blocks: ragged pulsars, Philox normals, both
    phiinv layouts (GS_OPT_PHI_PER_CHAIN), with and without a chain gate; all 45 pulsars (nm up to
    17: the fixed block stays row-major), only those with nm <= 16 (the fixed block in tiles too),
    and NF = 40 (the other 20 columns fixed-prior: nm up to 37)."""
    from pulsar_timing_gibbsspec_amd import _lib, synthetic
    from pulsar_timing_gibbsspec_amd.engine import DeviceModel
    pta = synthetic.array_pta(kind="curn", seed=0)
    T, N, R = pta.get_basis(), pta.get_ndiag({}), pta.get_residuals()
    keep = [p for p in range(len(T)) if not small_nm or T[p].shape[1] - nf <= 16]
    assert len(keep) >= 2
    T, N, R = [T[p] for p in keep], [N[p] for p in keep], [R[p] for p in keep]
    gwid = [np.arange(nf) for _ in T]
    model = DeviceModel(ctx, T, N, R, gwid, [np.full(T[p].shape[1] - nf, 1e-40) for p in range(len(T))])
    assert (model.NMX <= 16) == small_nm
    assert model.model_tiled is not None
    C = 37                                                  # ragged last chain group
    rng = np.random.default_rng(5)
    rows = C if phi_shared else model.P * C
    phi = dev(10.0 ** rng.uniform(12, 16, (rows, model.NF)))
    mask = dev((rng.uniform(size=C) < 0.7).astype(np.int32), torch.int32) if masked else None
    lib, h = ctx.lib, ctx.handle
    prev = ctx.get_option(_lib.OPT_PHI_PER_CHAIN)
    ctx.set_option(_lib.OPT_PHI_PER_CHAIN, int(phi_shared))
    out = []
    try:
        for fn, mb in ((lib.gs_bdraw, model.model), (lib.gs_bdraw_tiled, model.model_tiled)):
            b = torch.full((model.P * C, model.ldb), 7.0, dtype=torch.float64, device="cuda")
            info = torch.zeros(model.P * C, dtype=torch.int32, device="cuda")
            _lib.check(fn(h, model.P, C, model.NF, model.NMX, model.ldb, _lib.ptr(mb), _lib.ptr(model.fidx),
                          _lib.ptr(model.midx), _lib.ptr(model.nm_dev), _lib.ptr(phi), None, 3, _lib.EV_B, 0,
                          _lib.ptr(mask), _lib.ptr(b), _lib.ptr(info)), "bdraw")
            out.append((b.cpu().numpy(), info.cpu().numpy()))
    finally:
        ctx.set_option(_lib.OPT_PHI_PER_CHAIN, prev)
    (b0, i0), (b1, i1) = out
    assert not i0.any() and not i1.any()
    assert np.array_equal(b0, b1)
    if masked:                                              # gated systems keep b
        keep = np.tile(mask.cpu().numpy() == 0, model.P)
        assert keep.any() and np.all(b1[keep] == 7.0)


@pytest.mark.parametrize("ngrid", [1000, 1024, 333, 64, 1])
def test_curn_sum_certified_f32_matches_f64(ctx, request, ngrid):
    """The default CURN-from-sums draw (k_rho_curn_sum_cert16: f32 points relative to the row's
    mode + per-row error certificate, f64 redo of unproven rows) against the f64 wave kernel
    (GS_OPT_GRID_EXACT = 2) on 15k rows whose mode spans the grid and beyond it on both sides,
    with adversarial rows (u placed exactly on an f64 cdf value): the same index on every row, the
    adversarial ones among the few redone in f64."""
    from pulsar_timing_gibbsspec_amd import _lib
    from pulsar_timing_gibbsspec_amd.engine import grid3
    request.addfinalizer(lambda: ctx.lib.gs_ctx_set_option(ctx.handle, _lib.OPT_GRID_EXACT, 0))
    rng = np.random.default_rng(ngrid)
    P, n_f, C = 45, 30, 512
    lo, hi = 1e-18, 1e-8
    rho_true = 10 ** rng.uniform(-21, -5, (n_f, C))
    S = 2 * rho_true * rng.gamma(P, 1.0, (n_f, C))
    S[0, :8] = 0.0                                   # no data: pdf ~ rho^-P, the left edge
    u = rng.random((C, n_f))
    G = grid3(lo, hi, n=ngrid)
    rho = 10 ** np.linspace(np.log10(lo), np.log10(hi), ngrid)
    adv = list(zip(rng.integers(0, n_f, 40), rng.integers(8, C, 40)))
    for k, c in adv:
        lp = -P * np.log(rho) - S[k, c] / (2 * rho)
        cdf = np.cumsum(np.exp(lp - lp.max()))
        cdf /= cdf[-1]
        u[c, k] = cdf[int(rng.integers(0, ngrid))]
    xcol = torch.arange(n_f, dtype=torch.int32, device="cuda")
    fb = torch.zeros(1, dtype=torch.int32, device="cuda")
    out, nfb = {}, {}
    for mode in (2, 0):
        _lib.check(ctx.lib.gs_ctx_set_option(ctx.handle, _lib.OPT_GRID_EXACT, mode), "set_option")
        x = torch.zeros(C, n_f, dtype=torch.float64, device="cuda")
        idx = torch.full((n_f * C,), -7, dtype=torch.int32, device="cuda")
        K = Keep()
        fb.zero_()
        _lib.check(ctx.lib.gs_ctx_set_grid_fallback_counter(ctx.handle, _lib.ptr(fb)), "counter")
        try:
            _lib.check(ctx.lib.gs_rho_curn_sum(ctx.handle, P, C, n_f, K(S), ngrid, _lib.ptr(G), K(u), 0, 0,
                                               _lib.ptr(x), n_f, _lib.ptr(xcol), _lib.ptr(idx)), "gs_rho_curn_sum")
        finally:
            _lib.check(ctx.lib.gs_ctx_set_grid_fallback_counter(ctx.handle, None), "counter")
        out[mode] = (idx.cpu().numpy(), x.cpu().numpy())
        nfb[mode] = int(fb)
    assert out[0][0].min() >= 0 and out[0][0].max() < ngrid
    assert np.array_equal(out[0][0], out[2][0]), int(np.sum(out[0][0] != out[2][0]))
    assert np.array_equal(out[0][1], out[2][1])
    if ngrid > 1:
        assert nfb[0] < 0.03 * out[0][0].size, nfb[0]
