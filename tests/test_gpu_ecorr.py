""" Basis ECORR on the GPU, through the C-ABI, against the reference's own run
(tests/golden/ecorr_mh_j1713.npz: PulsarBlockGibbs.update_ecorr_params on its
get_lnlikelihood_fullmarg inside the notebook sampler's sweep order, every draw captured;
tests/golden/ecorr_long_j1713.npz: a long reference chain).

* marginalised likelihood at prior draws: |device - reference| < 1e-7 (values ~7e3; the
  device eliminates the diagonal epoch block first, the reference factors all 212 columns);
* the Metropolis block fed the reference's draws: accept/reject decisions coincide, so the
  ECORR parameters come out bit-identical;
* b | rho: the zero-normal draw is the conditional mean (1e-9 normwise vs the oracle's block
  form, 1e-8 vs a dense solve) and the normal -> b map G satisfies G^T Sigma G = I;
* the sampler (Philox draws, many chains): per-parameter KS test against the reference chain.
"""
import numpy as np
import pytest

from tests.conftest import golden, gpu_available
from oracle import gibbs_oracle as O
from tests.parity_data import normwise_rel

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    if not gpu_available():
        pytest.skip("no GPU")
    from pulsar_timing_gibbsspec_amd import _lib
    return _lib.Context(0, seed=11)


def _items(g):
    kinds, vals, lens = g["kinds"], g["vals"], g["lens"]
    off = np.concatenate([[0], np.cumsum(lens)])
    return [(kinds[i], vals[off[i]:off[i + 1]]) for i in range(kinds.size)]


def _model(ctx, g, C):
    from pulsar_timing_gibbsspec_amd.ecorr import EcorrModel
    eind = np.asarray(g["eind"])
    return EcorrModel(ctx, g["T"], g["Nvec"], g["r"], g["ecid"], g["epoch_backend"], g["gwid"], eind,
                      g["pmin"][eind], g["pmax"][eind], len(g["param_names"]), C)


def _gwind(g):
    return np.array([i for i, n in enumerate(g["param_names"]) if "rho" in n])


def _dev(a, dtype=None):
    import torch
    return torch.as_tensor(np.ascontiguousarray(a), dtype=dtype or torch.float64, device="cuda")


def _phiinv_F(g, X):
    return 1.0 / np.repeat(10.0 ** (2.0 * X[:, _gwind(g)]), 2, axis=1)


@pytest.mark.parametrize("mode", ["lnl", "block", "unfused"])
def test_ecorr_lnlike_matches_reference(ctx, mode):
    """The three device forms -- gs_ecorr_prefix in likelihood mode; gs_ecorr_prefix model
    block + gs_lnlike_marg; gs_ecorr_schur + gs_prefix_sys + gs_lnlike_marg -- against the
    reference's get_lnlikelihood_fullmarg, and the two model blocks against each other."""
    g = golden("ecorr_mh_j1713.npz")
    X = g["x_like"]
    em = _model(ctx, g, X.shape[0])
    assert em.fused
    fused = mode != "unfused"
    em.fused = fused
    em.fused_lnl = mode == "lnl"
    got = em.lnlike(_dev(X), _dev(_phiinv_F(g, X))).cpu().numpy()
    err = np.abs(got - g["lnlike"])
    assert err.max() < 1e-7, (got, g["lnlike"])
    if fused:
        em.factor(_dev(X), fused=True)
        a = em.model.clone()
        em.factor(_dev(X), fused=False)
        b = em.model
        NF, NMX = em.NF, em.NMX
        sizes = [NF * (NF + 1), NF, NMX * (NF + 1), NMX, NMX * NMX, 2]
        cut = np.cumsum(sizes)[:-1]
        A = a.view(X.shape[0], -1).cpu().numpy()[:, :sum(sizes)]
        B = b.view(X.shape[0], -1).cpu().numpy()[:, :sum(sizes)]
        for sa, sb in zip(np.split(A, cut, axis=1), np.split(B, cut, axis=1)):
            assert normwise_rel(sa, sb) < 1e-9


def test_ecorr_mh_matches_reference(ctx):
    """Every sweep's ECORR block of the reference run, one chain per sweep, fed the
    reference's (scale, parameter, normal, uniform) draws: outputs bit-identical."""
    g = golden("ecorr_mh_j1713.npz")
    eind = list(np.asarray(g["eind"]))
    acl = int(g["aclength"])
    n = g["e_in"].shape[0]
    items = iter(_items(g))
    inj = np.zeros((acl, n, 4))
    for ii in range(n):
        if ii == 0:
            assert next(items)[0] == "randn"      # first b
        for s in range(acl):
            (k1, sc), (k2, p), (k3, z), (k4, u) = next(items), next(items), next(items), next(items)
            assert (k1, k2, k3, k4) == ("choice", "choice", "randn", "rand")
            inj[s, ii] = (sc[0], eind.index(int(p[0])), z[0], u[0])
        assert next(items)[0] == "uniform"       # rho|b
        k, _ = next(items)                       # gated b
        assert k == "randn"
    em = _model(ctx, g, n)
    x = _dev(g["e_in"])
    import torch
    n_acc = torch.zeros(n, dtype=torch.int32, device="cuda")
    em.mh(x, _dev(_phiinv_F(g, g["e_in"])), acl, inj=_dev(inj), n_acc=n_acc)
    out = x.cpu().numpy()
    assert np.array_equal(out, g["e_out"]), np.abs(out - g["e_out"]).max()
    assert n_acc.cpu().numpy().min() > 0


def test_ecorr_bdraw_is_exact_conditional(ctx):
    import torch
    g = golden("ecorr_mh_j1713.npz")
    T, N, r = g["T"], g["Nvec"], g["r"]
    TNT, d = O.tnt(T, N, r)
    m = T.shape[1]
    x0 = g["x0"]
    eind, ecid, ebk, gwid = g["eind"], g["ecid"], g["epoch_backend"], g["gwid"]
    ph = np.full(m, 1e40)
    ph[ecid] = np.array([10.0 ** (2.0 * float(x0[e])) for e in eind])[ebk]
    ph[gwid] = np.repeat(10.0 ** (2.0 * x0[_gwind(g)]), 2)
    phiinv = 1.0 / ph
    C = m + 1
    em = _model(ctx, g, C)
    X = np.broadcast_to(x0, (C, x0.size))
    Z = np.zeros((C, m))
    Z[1:] = np.eye(m)
    b = torch.zeros(C, m, dtype=torch.float64, device="cuda")
    em.bdraw(_dev(X), _dev(_phiinv_F(g, X)), b, z=_dev(Z))
    B = b.cpu().numpy()
    rc = np.setdiff1d(np.arange(m), ecid)
    mean_o = O.bdraw_ecorr(TNT, d, ecid, phiinv, np.zeros(rc.size), np.zeros(ecid.size))
    assert normwise_rel(B[0], mean_o) < 1e-9
    Sig = TNT + np.diag(phiinv)
    assert normwise_rel(B[0], np.linalg.solve(Sig, d)) < 1e-8
    G = (B[1:] - B[0]).T
    assert np.abs(G.T @ Sig @ G - np.eye(m)).max() < 1e-6
    assert int(em.binfo.max()) == 0


def test_ecorr_sampler_posterior_ks(ctx):
    """Device sampler (Philox) vs the reference's long chain: per-parameter two-sample KS on
    the ECORR parameters and every log10_rho bin (reference thinned to ~independent draws)."""
    import torch
    from scipy.stats import ks_2samp
    from pulsar_timing_gibbsspec_amd.ecorr import EcorrFreeSpectrumChains
    g = golden("ecorr_mh_j1713.npz")
    L = golden("ecorr_long_j1713.npz")
    C, n_sweep, burn = 1024, 60, 40
    em = _model(ctx, g, C)
    run = EcorrFreeSpectrumChains(em, _gwind(g), g["gwid"], float(g["rhomin"]), float(g["rhomax"]),
                                  L["x0"], int(L["aclength"]))
    x_rec = torch.empty(n_sweep, C, len(g["param_names"]), dtype=torch.float64, device="cuda")
    for ii in range(n_sweep):
        run.sweep(x_rec=x_rec[ii])
    dev = x_rec[burn:].cpu().numpy()
    assert np.isfinite(dev).all()
    ref = L["chain"][200:]        # thinned by 5, burn-in 1000 sweeps
    ref = ref[::5]
    pmin = 1.0
    for j in list(np.asarray(g["eind"])) + list(_gwind(g)):
        p = ks_2samp(dev[-1, :, j], ref[:, j]).pvalue
        pmin = min(pmin, p)
    # 32 tests: family-wise threshold
    assert pmin > 1e-4, pmin


def test_pulsar_block_gibbs_ecorr_surface(ctx, tmp_path):
    """PulsarBlockGibbs on the ECORR model: prior parsing (:111-118), the notebook's
    get_lnlikelihood, update_ecorr_params fed the reference's first-sweep draws, and a
    short multi-chain sample() through the warm-up (chain files, finite rows)."""
    from pulsar_timing_gibbsspec_amd import synthetic
    from pulsar_timing_gibbsspec_amd.pulsar_gibbs import PulsarBlockGibbs
    g = golden("ecorr_mh_j1713.npz")
    pta = synthetic.ecorr_pulsar_pta("J1713+0747", seed=0)
    gb = PulsarBlockGibbs(pta, nchains=64, seed=3)
    assert np.allclose([gb.ecorrmin, gb.ecorrmax], [g["ecorrmin"], g["ecorrmax"]], rtol=0, atol=0)
    assert np.array_equal(gb.ecid, g["ecid"]) and np.array_equal(gb.gwid, g["gwid"])
    for x, ref in zip(g["x_like"], g["lnlike"]):
        assert abs(gb.get_lnlikelihood(x) - ref) < 1e-7
    eind = list(np.asarray(g["eind"]))
    items = iter(_items(g))
    assert next(items)[0] == "randn"
    acl = int(g["aclength"])
    inj = []
    for _ in range(acl):
        (_, sc), (_, p), (_, z), (_, u) = next(items), next(items), next(items), next(items)
        inj.append((sc[0], eind.index(int(p[0])), z[0], u[0]))
    gb.aclength_ecorr = acl
    assert np.array_equal(gb.update_ecorr_params(g["e_in"][0], inj=np.array(inj)), g["e_out"][0])
    del gb.aclength_ecorr
    chain = gb.sample(g["x0"], outdir=str(tmp_path), niter=12, save_every=5)
    assert chain.shape == (12, len(g["param_names"])) and np.isfinite(chain).all()
    assert gb.chains.shape[0] == 64 and 1 <= gb.aclength_ecorr < 1000
    assert np.load(tmp_path / "chain.npy").shape[0] == 11


# ----------------------------------------------------------------- white noise + ECORR
def _white_setup(ctx, g, C):
    from pulsar_timing_gibbsspec_amd.ecorr import EcorrModel
    from pulsar_timing_gibbsspec_amd.white import WhiteNoiseModel
    names = list(g["param_names"])
    wind, eind = list(np.asarray(g["wind"])), np.asarray(g["eind"])
    wl = []
    for j in wind:
        k = int(names[j].split("_b")[1].split("_")[0])
        kind = 0 if names[j].endswith("efac") else 1
        wl.append((int(j), kind, k, float(g["pmin"][j]), float(g["pmax"][j])))
    T, gwid = g["T"], np.asarray(g["gwid"])
    m = T.shape[1]
    wm = WhiteNoiseModel(ctx, [T], [g["r"]], [g["sigma"]], [g["backends"]], [gwid], [np.full(m - gwid.size, 1e-40)],
                         [wl], C, prefix=False)
    em = EcorrModel(ctx, T, g["sigma"] ** 2, g["r"], g["ecid"], g["epoch_backend"], gwid, eind, g["pmin"][eind],
                    g["pmax"][eind], len(names), C, per_chain=True)
    return wm, em, wind, eind


def _white_N(g, x):
    names = list(g["param_names"])
    bk = np.asarray(g["backends"])
    nb = int(bk.max()) + 1
    ef = np.array([x[names.index(f"J1713+0747_b{k}_efac")] for k in range(nb)])
    eq = np.array([10.0 ** (2.0 * float(x[names.index(f"J1713+0747_b{k}_log10_tnequad")])) for k in range(nb)])
    return ef[bk] ** 2 * g["sigma"] ** 2 + eq[bk]


def test_ecorr_white_lnlike_matches_reference(ctx):
    """Per-chain N (white parameters vary): gs_white_tnt -> gs_ecorr_gather -> likelihood-mode
    gs_ecorr_prefix against the reference's get_lnlikelihood_fullmarg at prior draws."""
    import torch
    g = golden("ecorr_white_j1713.npz")
    X = g["x_like"]
    C = X.shape[0]
    wm, em, _, _ = _white_setup(ctx, g, C)
    x = _dev(X)
    wm.tnt(x, x.shape[1])
    em.gather(wm.TNT, wm.d, wm.tnt_cstride, wm.d_cstride)
    r = g["r"]
    const = []
    for xx in X:
        N = _white_N(g, xx)
        const.append(-0.5 * (np.sum(np.log(N)) + np.sum(r ** 2 / N)) + 0.5 * em.nm * np.log(1e-40))
    got = em.lnlike(x, _dev(_phiinv_F(g, X)), lnl_const=torch.as_tensor(const, device="cuda")).cpu().numpy()
    assert np.abs(got - g["lnlike"]).max() < 1e-7, (got, g["lnlike"])


def test_ecorr_white_blocks_match_reference(ctx):
    """Sweeps 1.. of the reference's white + ECORR run, one chain per sweep, fed the reference's
    MH draws: the white block (on y = r - T b with the sweep's b) and then the ECORR block (on
    the chain's new N) reproduce the reference's outputs bit for bit."""
    import torch
    g = golden("ecorr_white_j1713.npz")
    wind, eind = list(np.asarray(g["wind"])), list(np.asarray(g["eind"]))
    aw, ae = int(g["aclength_white"]), int(g["aclength_ecorr"])
    n = g["w_in"].shape[0]
    items = iter(_items(g))
    iw = np.zeros((aw, n, 4))
    ie = np.zeros((ae, n, 4))
    for ii in range(n):
        if ii == 0:
            assert next(items)[0] == "randn"
        for s in range(aw):
            (k1, sc), (k2, p), (k3, z), (k4, u) = next(items), next(items), next(items), next(items)
            assert (k1, k2, k3, k4) == ("choice", "choice", "randn", "rand")
            iw[s, ii] = (sc[0], wind.index(int(p[0])), z[0], u[0])
        for s in range(ae):
            (k1, sc), (k2, p), (k3, z), (k4, u) = next(items), next(items), next(items), next(items)
            assert (k1, k2, k3, k4) == ("choice", "choice", "randn", "rand")
            ie[s, ii] = (sc[0], eind.index(int(p[0])), z[0], u[0])
        assert next(items)[0] == "uniform"
        assert next(items)[0] == "randn"
    sel = np.arange(1, n)          # sweep 0's white block used the unrecorded first b
    C = sel.size
    wm, em, _, _ = _white_setup(ctx, g, C)
    x = _dev(g["w_in"][sel])
    b = _dev(g["bhist"][sel])
    wm.resid(b)
    wm.mh(x, x.shape[1], aw, 0, inj=_dev(iw[:, sel]))
    assert np.array_equal(x.cpu().numpy(), g["w_out"][sel])
    wm.tnt(x, x.shape[1])
    em.gather(wm.TNT, wm.d, wm.tnt_cstride, wm.d_cstride)
    em.mh(x, _dev(_phiinv_F(g, g["w_out"][sel])), ae, inj=_dev(ie[:, sel]))
    assert np.array_equal(x.cpu().numpy(), g["e_out"][sel])


def test_ecorr_white_operand_routes_agree(ctx):
    """Per-chain ECORR operands two ways: the full m x m SYRK (gs_white_tnt) + gs_ecorr_gather,
    and the R-column SYRK + epoch segment sums (gs_ecorr_epoch_sums) -- equal to 1e-12."""
    import torch
    from pulsar_timing_gibbsspec_amd.ecorr import EcorrWhiteChains, white_ecorr_models
    g = golden("ecorr_white_j1713.npz")
    X = g["x_like"]
    C = X.shape[0]
    _, _, wind, eind = _white_setup(ctx, g, 1)
    names = list(g["param_names"])
    wl = [(int(j), 0 if names[j].endswith("efac") else 1, int(names[j].split("_b")[1].split("_")[0]),
           float(g["pmin"][j]), float(g["pmax"][j])) for j in wind]
    wm, wmR, em = white_ecorr_models(ctx, g["T"], g["r"], g["sigma"], g["backends"], g["gwid"], wl, g["ecid"],
                                     g["epoch_backend"], eind, g["pmin"][eind], g["pmax"][eind], len(names), C)
    run = EcorrWhiteChains(wm, em, _gwind(g), g["gwid"], float(g["rhomin"]), float(g["rhomax"]), X[0], 1, 1,
                           wmR=wmR)
    run.x.copy_(_dev(X))
    run._operands()
    A = [t.clone().cpu().numpy() for t in (em.Bp, em.Dg, em.Ap)]
    run.wmR = None
    run._operands()
    B = [t.cpu().numpy() for t in (em.Bp, em.Dg, em.Ap)]
    for a, b in zip(A, B):
        a, b = a.reshape(C, -1), b.reshape(C, -1)
        assert normwise_rel(a, b) < 1e-12, normwise_rel(a, b)


def test_ecorr_white_sampler_runs(ctx):
    """Philox sampler with both blocks, 256 chains: finite chains, both blocks accept, and
    the per-chain b draw is the exact conditional mean at zero normals."""
    import torch
    from pulsar_timing_gibbsspec_amd.ecorr import EcorrWhiteChains
    g = golden("ecorr_white_j1713.npz")
    C = 256
    wm, em, _, _ = _white_setup(ctx, g, C)
    run = EcorrWhiteChains(wm, em, _gwind(g), g["gwid"], float(g["rhomin"]), float(g["rhomax"]), g["x0"], 10, 10)
    x_rec = torch.empty(12, C, len(g["param_names"]), dtype=torch.float64, device="cuda")
    for ii in range(12):
        run.sweep(x_rec=x_rec[ii])
    X = x_rec.cpu().numpy()
    assert np.isfinite(X).all() and np.isfinite(run.b.cpu().numpy()).all()
    assert run.n_acc_white.min().item() > 0 and run.n_acc_ecorr.min().item() > 0
    assert int(em.pinfo.abs().max()) == 0 and int(em.binfo.abs().max()) == 0
    # exact conditional mean at chain 0's state (zero normals)
    x0 = run.x[:1].expand(C, -1).contiguous()
    run.x.copy_(x0)
    run._operands()
    run._phiinv(False)
    bz = torch.zeros(C, em.m, dtype=torch.float64, device="cuda")
    em.bdraw(run.x, run.phiinv_F, bz, z=torch.zeros(C, em.m, dtype=torch.float64, device="cuda"))
    xx = run.x[0].cpu().numpy()
    N = _white_N(g, xx)
    TNT, d = O.tnt(g["T"], N, g["r"])
    m = em.m
    ph = np.full(m, 1e40)
    ph[np.asarray(g["ecid"])] = np.array([10.0 ** (2 * float(xx[e])) for e in g["eind"]])[g["epoch_backend"]]
    ph[np.asarray(g["gwid"])] = np.repeat(10.0 ** (2 * xx[_gwind(g)]), 2)
    ref = np.linalg.solve(TNT + np.diag(1.0 / ph), d)
    assert normwise_rel(bz[0].cpu().numpy(), ref) < 1e-8


def test_pulsar_block_gibbs_ecorr_white_surface(ctx, tmp_path):
    """PulsarBlockGibbs with white noise and ECORR sampled: get_lnlikelihood at prior draws of
    every parameter (white included) against the reference, update_white_params followed by
    update_ecorr_params on the reference's sweep-1 draws, and a short multi-chain sample()."""
    from pulsar_timing_gibbsspec_amd import synthetic
    from pulsar_timing_gibbsspec_amd.pulsar_gibbs import PulsarBlockGibbs
    g = golden("ecorr_white_j1713.npz")
    pta = synthetic.ecorr_pulsar_pta("J1713+0747", seed=0, white_vary=True)
    gb = PulsarBlockGibbs(pta, nchains=32, seed=5)
    for x, ref in zip(g["x_like"], g["lnlike"]):
        assert abs(gb.get_lnlikelihood(x) - ref) < 1e-7
    wind, eind = list(np.asarray(g["wind"])), list(np.asarray(g["eind"]))
    aw, ae = int(g["aclength_white"]), int(g["aclength_ecorr"])
    items = iter(_items(g))
    assert next(items)[0] == "randn"
    for _ in range(aw + ae):          # sweep 0
        next(items), next(items), next(items), next(items)
    next(items), next(items)
    iw, ie = [], []
    for _ in range(aw):
        (_, sc), (_, p), (_, z), (_, u) = next(items), next(items), next(items), next(items)
        iw.append((sc[0], wind.index(int(p[0])), z[0], u[0]))
    for _ in range(ae):
        (_, sc), (_, p), (_, z), (_, u) = next(items), next(items), next(items), next(items)
        ie.append((sc[0], eind.index(int(p[0])), z[0], u[0]))
    gb.aclength_white, gb.aclength_ecorr = aw, ae
    gb._b = g["bhist"][1]
    xw = gb.update_white_params(g["w_in"][1], inj=np.array(iw))
    assert np.array_equal(xw, g["w_out"][1])
    assert np.array_equal(gb.update_ecorr_params(xw, inj=np.array(ie)), g["e_out"][1])
    del gb.aclength_white, gb.aclength_ecorr
    gb._b = np.zeros_like(gb._b)
    chain = gb.sample(g["x0"], outdir=str(tmp_path), niter=8, save_every=4)
    assert chain.shape == (8, len(g["param_names"])) and np.isfinite(chain).all()
    assert gb.chains.shape[0] == 32 and gb.aclength_white >= 1 and gb.aclength_ecorr >= 1


def test_ecorr_bdraw_chain_mask_mixed(ctx):
    """the 8-chain shared-Bx b_E kernel (k_ecorr_bdraw_e<8>) with a mixed 0/1
    chain_mask and n_chain not a multiple of 8: masked chains keep their b untouched (both
    the b_R draw and the b_E scatter), unmasked chains equal the same draw run unmasked."""
    import torch
    g = golden("ecorr_mh_j1713.npz")
    m = g["T"].shape[1]
    C = 13
    em = _model(ctx, g, C)
    rng = np.random.default_rng(5)
    X = np.broadcast_to(g["x0"], (C, g["x0"].size)).copy()
    X[:, _gwind(g)] += rng.uniform(-0.3, 0.3, (C, len(_gwind(g))))
    Z = rng.standard_normal((C, m))
    ref = torch.zeros(C, m, dtype=torch.float64, device="cuda")
    em.bdraw(_dev(X), _dev(_phiinv_F(g, X)), ref, z=_dev(Z))
    mask = np.array([1, 0, 1, 1, 0, 0, 1, 0, 1, 1, 1, 0, 1], np.int32)
    sentinel = 123.25
    b = torch.full((C, m), sentinel, dtype=torch.float64, device="cuda")
    em.bdraw(_dev(X), _dev(_phiinv_F(g, X)), b, z=_dev(Z), chain_mask=torch.as_tensor(mask, device="cuda"))
    B, R = b.cpu().numpy(), ref.cpu().numpy()
    for c in range(C):
        if mask[c]:
            assert np.array_equal(B[c], R[c]), c
        else:
            assert np.all(B[c] == sentinel), c


@pytest.mark.parametrize("mR,ne,offset", [(60, 137, 0), (100, 137, 0), (120, 137, 0), (60, 1, 1), (76, 33, 1),
                                           (100, 64, 1)])
def test_ecorr_schur_direct(ctx, mR, ne, offset):
    """gs_ecorr_schur through the C-ABI on random operands: TNT = A - B^T diag(1/a) B,
    d = dR - B^T (d_E / a), aux = (sum log a, sum d_E^2 / a, sum log phi_E, 0), against
    numpy.  mR = 100 / 120 use 7 / 8 tile columns, whose accumulators are split over two
    launches (one would need ~290 VGPRs).  offset = 1: Bx at an 8-byte offset address (the LDS-DMA
    staging in 4-byte units); ne = 1 / 33 / 64: partial and exact 32-epoch chunks."""
    import torch
    from pulsar_timing_gibbsspec_amd._lib import check, ptr
    rng = np.random.default_rng(mR + ne)
    C, n_bk = 5, 3
    ldbx = 16 * ((mR + 16) // 16)
    Bx = np.zeros((ne, ldbx))
    Bx[:, :mR + 1] = rng.standard_normal((ne, mR + 1))
    Dg = rng.uniform(0.5, 2.0, ne)
    ebk = rng.integers(0, n_bk, ne).astype(np.int32)
    ldx = 7
    x = rng.uniform(-1.0, 0.5, (C, ldx))
    xcol = np.array([1, 3, 6], np.int32)
    Araw = rng.standard_normal((mR, mR))
    A = Araw @ Araw.T + mR * np.eye(mR)
    dR = rng.standard_normal(mR)
    dev = lambda a, dt=torch.float64: torch.as_tensor(np.ascontiguousarray(a), dtype=dt, device=ctx.device)  # noqa: E731
    g = {k: dev(v) for k, v in dict(Bx=Bx, Dg=Dg, x=x, A=A, dR=dR).items()}
    g["ebk"], g["xcol"] = dev(ebk, torch.int32), dev(xcol, torch.int32)
    if offset:
        buf = torch.zeros(Bx.size + 1, dtype=torch.float64, device=ctx.device)
        buf[1:] = g["Bx"].reshape(-1)
        g["Bx"] = buf[1:]
        assert g["Bx"].data_ptr() % 16 == 8
    TNT = torch.empty(C, mR, mR, dtype=torch.float64, device=ctx.device)
    d = torch.empty(C, mR, dtype=torch.float64, device=ctx.device)
    aux = torch.empty(C, 4, dtype=torch.float64, device=ctx.device)
    check(ctx.lib.gs_ecorr_schur(ctx.handle, C, mR, ne, ldbx, ptr(g["Bx"]), ptr(g["Dg"]), ptr(g["ebk"]), n_bk,
                                 ptr(g["xcol"]), ptr(g["x"]), ldx, ptr(g["A"]), ptr(g["dR"]), ptr(TNT), ptr(d),
                                 ptr(aux)), "gs_ecorr_schur")
    TNT, d, aux = TNT.cpu().numpy(), d.cpu().numpy(), aux.cpu().numpy()
    B, dE = Bx[:, :mR], Bx[:, mR]
    for c in range(C):
        ph = 10.0 ** (2.0 * x[c, xcol])
        a = Dg + 1.0 / ph[ebk]
        want = A - B.T @ (B / a[:, None])
        assert np.max(np.abs(TNT[c] - want)) <= 1e-12 * np.max(np.abs(want)), (mR, c)
        assert np.array_equal(TNT[c], TNT[c].T)
        assert normwise_rel(d[c], dR - B.T @ (dE / a)) < 1e-12
        np.testing.assert_allclose(aux[c, :3], [np.sum(np.log(a)), np.sum(dE ** 2 / a), np.sum(np.log(ph[ebk]))],
                                   rtol=1e-12)
        assert aux[c, 3] == 0.0


@pytest.mark.parametrize("n_tm", [40, 56])
def test_ecorr_lnlike_wide_timing_model(ctx, n_tm):
    """PulsarBlockGibbs.get_lnlikelihood on ECORR models whose R block (60 free-spectrum + n_tm
    timing-model columns, m_R = 100 / 116) needs 7 / 8 Schur tile columns (the split launches):
    against the oracle's get_lnlikelihood_fullmarg restatement (pulsar_gibbs.py:569-610)."""
    from pulsar_timing_gibbsspec_amd import synthetic
    from pulsar_timing_gibbsspec_amd.pulsar_gibbs import PulsarBlockGibbs
    pta = synthetic.ecorr_pulsar_pta("J1713+0747", seed=2, n_tm=n_tm)
    gb = PulsarBlockGibbs(pta, nchains=4, seed=3)
    T, r = pta.get_basis()[0], pta.get_residuals()[0]
    rng = np.random.default_rng(n_tm)
    for _ in range(3):
        x = np.concatenate([p.sample().flatten() for p in gb.params])
        x[gb.get_ecorr_indices()] = rng.uniform(-8.0, -5.5, len(gb.get_ecorr_indices()))
        params = gb.map_params(x)
        N = pta.get_ndiag(params)[0]
        phiinv, logdet = pta.get_phiinv(params, logdet=True)[0]
        TNT, d = O.tnt(T, N, r)
        ref = O.lnlike_fullmarg(r, N, TNT, d, phiinv, logdet)
        got = gb.get_lnlikelihood(x)
        assert gb._em1.mR == 60 + n_tm and not gb._em1.fused
        assert abs(got - ref) < 1e-7 * max(1.0, abs(ref)), (n_tm, got, ref)


def _prefix_lnl_numpy(Bp, Dg, ebk, Ap, xrow, ecol, phiinv_F, NF):
    """Likelihood-mode gs_ecorr_prefix outputs from its operands (the [M (16) | F | d | pad]
    layout): T = Ap - Bp^T diag(1/a) Bp, Sigma = T_RR + diag(0_M, phiinv_F), dd = T_Rd;
    lnl = (P_dd + dd^T Sigma^-1 dd - logdet Sigma + sum log phiinv_F) / 2, aux = (sum log a, 0,
    sum log phi_E, P_dd)."""
    ph = 10.0 ** (2.0 * xrow[ecol])
    a = Dg + 1.0 / ph[ebk]
    P = Bp.T @ (Bp / a[:, None])
    T = Ap - P
    R, dc = 16 + NF, 16 + NF
    S = T[:R, :R] + np.diag(np.concatenate([np.zeros(16), phiinv_F]))
    dd = T[:R, dc]
    quad = P[dc, dc] + dd @ np.linalg.solve(S, dd)
    lnl = 0.5 * (quad - np.linalg.slogdet(S)[1] + np.sum(np.log(phiinv_F)))
    return lnl, np.array([np.sum(np.log(a)), 0.0, np.sum(np.log(ph[ebk])), P[dc, dc]])


@pytest.mark.parametrize("ne", [1, 7, 64, 65, 136])
def test_ecorr_prefix_staging_edges(ctx, ne):
    """gs_ecorr_prefix (likelihood mode) on the first ne epochs of the J1713 operands, four ways:
    shared [B | d_E] at a 16-byte aligned and at an 8-byte offset address (LDS-DMA in 16- / 4-byte
    units), and per-chain copies with a chain stride of ne*KB (aligned) and ne*KB + 1 doubles
    (every other chain 8-byte offset) -- the lnl bit-identical across the four, and against numpy
    from the same operands to 1e-9 (ne = 1, 7: partial chunks; 64 / 65: the per-chain path's
    64-epoch weight segments)."""
    import torch
    from pulsar_timing_gibbsspec_amd._lib import check, ptr
    g = golden("ecorr_mh_j1713.npz")
    X = g["x_like"][:6]
    C = X.shape[0]
    em = _model(ctx, g, C)
    assert em.fused and not em.per_chain
    NF, KB = em.NF, em.ldbp
    Bp = em.Bp[:ne].contiguous()
    Dg, ebk = em.Dg[:ne].contiguous(), em.ebk[:ne].contiguous()
    Ap = em.Ap
    x = _dev(X)
    phf = _dev(_phiinv_F(g, X))
    Bn, Dn, En, An = Bp.cpu().numpy(), Dg.cpu().numpy(), ebk.cpu().numpy(), Ap.cpu().numpy()
    ecol = em.ecol.cpu().numpy()

    def run(Bx, Dgx, Apx, strides):
        lnl = torch.empty(C, dtype=torch.float64, device="cuda")
        aux = torch.empty(C, 4, dtype=torch.float64, device="cuda")
        info = torch.zeros(C, dtype=torch.int32, device="cuda")
        check(ctx.lib.gs_ecorr_prefix(ctx.handle, C, NF, em.NMX, em.nm, ne, KB, ptr(Bx), ptr(Dgx), ptr(ebk), em.n_bk,
                                      ptr(em.ecol), ptr(x), x.shape[1], ptr(Apx), ptr(phf), None, ptr(aux), ptr(lnl),
                                      ptr(info), *strides), "gs_ecorr_prefix")
        assert int(info.abs().max()) == 0
        return lnl.cpu().numpy(), aux.cpu().numpy()

    off = torch.zeros(ne * KB + 1, dtype=torch.float64, device="cuda")
    off[1:] = Bp.reshape(-1)
    assert off[1:].data_ptr() % 16 == 8
    outs = [run(Bp, Dg, Ap, (0, 0, 0)), run(off[1:], Dg, Ap, (0, 0, 0))]
    for extra in (0, 1):
        cs = ne * KB + extra
        Bc = torch.zeros(C * cs, dtype=torch.float64, device="cuda")
        for c in range(C):
            Bc[c * cs:c * cs + ne * KB] = Bp.reshape(-1)
        Dc = Dg.repeat(C).contiguous()
        Ac = Ap.reshape(1, -1).repeat(C, 1).contiguous()
        outs.append(run(Bc, Dc, Ac, (cs, ne, KB * KB)))
    for lnl, aux in outs[1:]:
        assert np.array_equal(lnl, outs[0][0])
        np.testing.assert_allclose(aux, outs[0][1], rtol=1e-13, atol=0)
    for c in range(C):
        want, waux = _prefix_lnl_numpy(Bn, Dn, En, An, X[c], ecol, _phiinv_F(g, X)[c], NF)
        assert abs(outs[0][0][c] - want) < 1e-9 * max(1.0, abs(want)), (ne, c, outs[0][0][c], want)
        np.testing.assert_allclose(outs[0][1][c], waux, rtol=1e-11, atol=1e-11)


def _mh_both_ways(em, x0, phf, n_steps, sweep=3):
    """em.mh from x0 with the incremental state steps and with a full evaluation per step (same
    Philox draws): (x, lnl0, n_acc) of each, and the stored state's deviation from a fresh T(x)."""
    import torch
    out = []
    for inc in (True, False):
        em.incremental = inc
        x = x0.clone()
        n_acc = torch.zeros(x.shape[0], dtype=torch.int32, device="cuda")
        em.mh(x, phf, n_steps, sweep=sweep, n_acc=n_acc)
        out.append((x.cpu().numpy(), em.lnl0.cpu().numpy().copy(), n_acc.cpu().numpy()))
        if inc:
            C = x.shape[0]
            cur = em.tbuf[em.tidx.long(), torch.arange(C, device="cuda")].clone()
            em.tidx.zero_()
            em._eval_state(x, phf)               # fresh full T(x) into slot 0
            fresh = em.tbuf[0].clone()
            dev = float(((cur - fresh).abs().amax(dim=1) / fresh.abs().amax(dim=1)).max())
    em.incremental = True
    return out, dev


def test_ecorr_incremental_steps_match_full(ctx):
    """The incremental Metropolis step (gs_ecorr_lnl_state: only the moved backend's epochs
    re-weighted from the stored T) against a full evaluation per step, 256 chains x 200 Philox steps
    (past one REFRESH): identical accept/reject decisions (x and acceptance counts bit-identical),
    lnL0 within 1e-9 relative, and the stored state within 1e-11 of a fresh T(x)."""
    g = golden("ecorr_mh_j1713.npz")
    C = 256
    X = np.repeat(g["x_like"][:1], C, axis=0)
    em = _model(ctx, g, C)
    assert em.eoff_host[0] == 0 and em.eoff_host[-1] == em.ne and np.all(np.diff(em.eoff_host) > 0)
    (a, b), dev = _mh_both_ways(em, _dev(X), _dev(_phiinv_F(g, X)), 200)
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[2], b[2])
    assert a[2].min() > 0
    np.testing.assert_allclose(a[1], b[1], rtol=1e-9, atol=0)
    assert dev < 1e-11, dev


def test_ecorr_white_incremental_steps_match_full(ctx):
    """The same with per-chain operands (white noise sampled: gs_white_tnt -> gs_ecorr_gather), the
    chains at different white-noise states."""
    g = golden("ecorr_white_j1713.npz")
    X = g["x_like"]
    C = X.shape[0]
    wm, em, _, _ = _white_setup(ctx, g, C)
    x = _dev(X)
    wm.tnt(x, x.shape[1])
    em.gather(wm.TNT, wm.d, wm.tnt_cstride, wm.d_cstride)
    (a, b), dev = _mh_both_ways(em, x, _dev(_phiinv_F(g, X)), 80)
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[2], b[2])
    np.testing.assert_allclose(a[1], b[1], rtol=1e-9, atol=0)
    assert dev < 1e-11, dev


def test_ecorr_four_backends_incremental_and_oracle(ctx):
    """Four backends, the epoch columns handed over in a shuffled order (EcorrModel groups them by
    backend for the incremental step): incremental vs full-evaluation Metropolis steps (identical
    decisions), and the likelihood at the chains' final states against the oracle's
    get_lnlikelihood_fullmarg restatement (pulsar_gibbs.py:569-610) on the full basis, to 1e-7."""
    import torch
    from pulsar_timing_gibbsspec_amd import synthetic
    from pulsar_timing_gibbsspec_amd.ecorr import EcorrModel
    from pulsar_timing_gibbsspec_amd.pulsar_gibbs import PulsarBlockGibbs
    pta = synthetic.ecorr_pulsar_pta("J1713+0747", seed=5, n_backends=4, n_epoch=120)
    names = pta.param_names
    ebk = pta.signals["J1713+0747_basis_ecorr"].epoch_backend
    ne = ebk.size
    perm = np.random.default_rng(3).permutation(ne)
    assert not np.all(np.diff(ebk[perm]) >= 0)
    eind = [i for i, n in enumerate(names) if "ecorr" in n]
    gw = [i for i, n in enumerate(names) if "rho" in n]
    T, r = pta.get_basis()[0], pta.get_residuals()[0]
    gwid = ne + np.arange(2 * len(gw))
    C = 128
    em = EcorrModel(ctx, T, pta.get_ndiag()[0], r, perm, ebk[perm], gwid, eind, [-8.5] * 4, [-5.0] * 4,
                    len(names), C)
    assert np.all(np.diff(em.ebk.cpu().numpy()) >= 0) and em.eoff_host.size == 5
    rng = np.random.default_rng(7)
    X = np.concatenate([rng.uniform(-7.5, -5.5, (C, len(eind))), rng.uniform(-8, -5, (C, len(gw)))], axis=1)
    phf = _dev(1.0 / np.repeat(10.0 ** (2.0 * X[:, gw]), 2, axis=1))
    (a, b), dev = _mh_both_ways(em, _dev(X), phf, 120)
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[2], b[2]) and a[2].min() > 0
    np.testing.assert_allclose(a[1], b[1], rtol=1e-9, atol=0)
    assert dev < 1e-11, dev
    Xf = a[0]
    got = em.lnlike(_dev(Xf), _dev(1.0 / np.repeat(10.0 ** (2.0 * Xf[:, gw]), 2, axis=1))).cpu().numpy()
    gb = PulsarBlockGibbs(pta, nchains=1, seed=0)
    for c in range(0, C, 37):
        params = gb.map_params(Xf[c])
        N = pta.get_ndiag(params)[0]
        phiinv, logdet = pta.get_phiinv(params, logdet=True)[0]
        TNT, d = O.tnt(T, N, r)
        ref = O.lnlike_fullmarg(r, N, TNT, d, phiinv, logdet)
        assert abs(got[c] - ref) < 1e-7 * max(1.0, abs(ref)), (c, got[c], ref)
