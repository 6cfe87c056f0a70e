"""Generate golden fixtures by running the REFERENCE sampler (this container only).

The reference tree (``/root/reference``) is imported read-only, with
``sys.dont_write_bytecode`` set, and only the vectors it produces are written
under ``tests/golden/``.  Three third-party modules it imports at module level
are absent here and are replaced by EMPTY module objects (``acor``,
``enterprise.signals.selections``, ``PTMCMCSampler.PTMCMCSampler.PTSampler``);
none of them is called on the paths exercised below.  The
enterprise PTA it consumes is our own facade (``pulsar_timing_gibbsspec_amd.synthetic``).

Every draw the reference makes from the global ``np.random`` is captured in
call order (``randn``, ``uniform`` as its underlying U(0,1) sample, ``gumbel``
as its underlying U(0,1) sample), so the oracle and the HIP path can be
replayed on exactly the same random numbers.

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py [/root/reference]
"""
import importlib.util
import os
import sys
import tempfile
import time
import types

os.environ.setdefault("OPENBLAS_NUM_THREADS", "1")
os.environ.setdefault("OMP_NUM_THREADS", "1")

import numpy as np  # noqa: E402

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.abspath(os.path.join(HERE, "..", "..")))

from pulsar_timing_gibbsspec_amd import synthetic  # noqa: E402


# ----------------------------------------------------------------- reference import
def _stub(name, **attrs):
    m = types.ModuleType(name)
    for k, v in attrs.items():
        setattr(m, k, v)
    sys.modules[name] = m
    return m


def load_reference(root):
    _stub("acor")
    ent = _stub("enterprise")
    sig = _stub("enterprise.signals")
    sel = _stub("enterprise.signals.selections")
    ent.signals = sig
    sig.selections = sel
    pt = _stub("PTMCMCSampler")
    ptm = _stub("PTMCMCSampler.PTMCMCSampler", PTSampler=object)
    pt.PTMCMCSampler = ptm
    mods = {}
    for name in ("pulsar_gibbs", "pta_gibbs"):
        spec = importlib.util.spec_from_file_location(f"_ref_{name}", os.path.join(root, name + ".py"))
        mod = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(mod)
        mods[name] = mod
    return mods


# ----------------------------------------------------------------- draw capture
class Capture:
    """Wrap np.random.{randn,uniform,gumbel}; record the unit draws in call order."""

    def __init__(self):
        self.log = []  # (kind, array)
        self._orig = {}

    def __enter__(self):
        R = np.random
        self._orig = dict(randn=R.randn, uniform=R.uniform, gumbel=R.gumbel, choice=R.choice, rand=R.rand)
        rs = R.random_sample
        cap = self

        def choice(a, size=None, replace=True, p=None):
            v = self._orig["choice"](a, size=size, replace=replace, p=p)
            cap.log.append(("choice", np.array(v, dtype=float)))
            return v

        def rand(*shape):
            v = self._orig["rand"](*shape)
            cap.log.append(("rand", np.array(v, dtype=float)))
            return v

        def randn(*shape):
            z = self._orig["randn"](*shape)
            cap.log.append(("randn", np.array(z, dtype=float)))
            return z

        def uniform(low=0.0, high=1.0, size=None):
            low_a, high_a = np.asarray(low, float), np.asarray(high, float)
            if size is None:
                size = np.broadcast(low_a, high_a).shape
            u = rs(size)
            cap.log.append(("uniform", np.array(u, dtype=float)))
            return low_a + (high_a - low_a) * u   # numpy: low + (high-low)*next_double

        def gumbel(loc=0.0, scale=1.0, size=None):
            u = rs(size)
            cap.log.append(("gumbel", np.array(u, dtype=float)))
            return loc - scale * np.log(-np.log1p(-u))   # numpy legacy gumbel

        R.randn, R.uniform, R.gumbel = randn, uniform, gumbel
        R.choice, R.rand = choice, rand
        return self

    def __exit__(self, *a):
        R = np.random
        R.randn, R.uniform, R.gumbel = (self._orig["randn"], self._orig["uniform"],
                                        self._orig["gumbel"])
        R.choice, R.rand = self._orig["choice"], self._orig["rand"]

    def take(self, kind):
        return [a for k, a in self.log if k == kind]


def _quiet(fn, *a, **k):
    import contextlib
    import io
    with contextlib.redirect_stdout(io.StringIO()), contextlib.redirect_stderr(io.StringIO()):
        return fn(*a, **k)


# ----------------------------------------------------------------- fixtures
def single_pulsar(ref, out, niter=300):
    """Config 1: J1713, 30-bin free spectrum, analytic rho|b (pulsar_gibbs.py:206-216)."""
    pta = synthetic.single_pulsar_pta("J1713+0747", seed=0)
    np.random.seed(1)
    g = _quiet(ref.PulsarBlockGibbs, pta)
    x0 = np.concatenate([p.sample().flatten() for p in g.params])
    T = pta.get_basis()[0]
    N = pta.get_ndiag({})[0]
    r = pta.get_residuals()[0]
    with tempfile.TemporaryDirectory() as d, Capture() as cap:
        np.random.seed(2)
        _quiet(g.sample, x0, outdir=d, niter=niter)
        saved_chain = np.load(os.path.join(d, "chain.npy"))
        saved_names = open(os.path.join(d, "pars_chain.txt")).read().split()
        saved_bnames = open(os.path.join(d, "pars_bchain.txt")).read().split()
    z = np.stack(cap.take("randn"))            # (niter+1, m): first draw + one per sweep
    U = np.stack(cap.take("uniform"))          # (niter, n_f)
    np.savez_compressed(out, T=T, Nvec=N, r=r, gwid=np.asarray(g.gwid), rhomin=g.rhomin,
                        rhomax=g.rhomax, x0=x0, z=z, U=U, chain=g.chain, bchain=g.bchain,
                        b_final=g._b, saved_rows=saved_chain.shape[0],
                        param_names=np.array(saved_names), b_param_names=np.array(saved_bnames))
    print("single:", out, z.shape, U.shape, saved_chain.shape)


def single_pulsar_long(ref, out, niter=40000, thin=10):
    """Long reference chain (independent draws) for the KS posterior comparison."""
    pta = synthetic.single_pulsar_pta("J1713+0747", seed=0)
    np.random.seed(11)
    g = _quiet(ref.PulsarBlockGibbs, pta)
    x0 = np.concatenate([p.sample().flatten() for p in g.params])
    with tempfile.TemporaryDirectory() as d:
        np.random.seed(12)
        _quiet(g.sample, x0, outdir=d, niter=niter)
    np.savez_compressed(out, chain=g.chain[::thin].astype(np.float32), thin=thin, niter=niter)
    print("long:", out, g.chain.shape)


def single_pulsar_gumbel(ref, out, ncalls=2):
    """Grid + Gumbel-max rho|b with intrinsic red noise present (pulsar_gibbs.py:222-234)."""
    pta = synthetic.single_pulsar_pta("J1713+0747", seed=0, powerlaw_red=True)
    np.random.seed(3)
    g = _quiet(ref.PulsarBlockGibbs, pta)
    x0 = np.concatenate([p.sample().flatten() for p in g.params])
    rs = np.random.RandomState(4)
    bs, xs, xnew, G = [], [], [], []
    for c in range(ncalls):
        b = rs.standard_normal(len(g._b)) * 10 ** rs.uniform(-8, -6.5, len(g._b))
        x = x0.copy()
        x[g.get_red_param_indices()] = [rs.uniform(-15, -13), rs.uniform(2, 5)]
        g._b = b
        with Capture() as cap:
            xn = g.update_gwrho_params(x)
        bs.append(b), xs.append(x), xnew.append(xn), G.append(cap.take("gumbel")[0])
    irn = [np.array(g.red_sig.get_phi(g.map_params(x)))[::2] for x in xs]
    np.savez_compressed(out, b=np.stack(bs), x=np.stack(xs), xnew=np.stack(xnew),
                        gumbel_u=np.stack(G), irn=np.stack(irn), gwid=np.asarray(g.gwid),
                        rhomin=g.rhomin, rhomax=g.rhomax,
                        gwind=g.get_gwrho_param_indices(), param_names=np.array(g.param_names))
    print("gumbel:", out)


def red_likelihood(ref, out, npts=16):
    """get_lnlikelihood_red (pulsar_gibbs.py:549-566) of the power-law red-noise model at
    random (b, log10_A, gamma, rho) points, plus the reference's log-probability gate
    inputs: the values the device red MH block must reproduce."""
    pta = synthetic.single_pulsar_pta("J1713+0747", seed=0, powerlaw_red=True)
    np.random.seed(5)
    g = _quiet(ref.PulsarBlockGibbs, pta)
    x0 = np.concatenate([p.sample().flatten() for p in g.params])
    rs = np.random.RandomState(6)
    rind = g.get_red_param_indices()
    names = list(g.param_names)
    ia = [i for i in rind if "log10_A" in names[i]][0]
    ig = [i for i in rind if "gamma" in names[i]][0]
    bs, xs, lnl, irn, gwphi = [], [], [], [], []
    for _ in range(npts):
        b = rs.standard_normal(len(g._b)) * 10 ** rs.uniform(-8, -6.5, len(g._b))
        x = x0.copy()
        x[g.get_gwrho_param_indices()] = rs.uniform(-9, -4, len(g.get_gwrho_param_indices()))
        x[ia], x[ig] = rs.uniform(-16, -12), rs.uniform(1, 6)
        g._b = b
        lnl.append(g.get_lnlikelihood_red(x))
        prm = g.map_params(x)
        irn.append(np.array(g.red_sig.get_phi(prm))[::2])
        gwphi.append(np.array(g.gw_sig.get_phi(prm))[::2])
        bs.append(b), xs.append(x)
    np.savez_compressed(out, b=np.stack(bs), x=np.stack(xs), lnl=np.array(lnl), irn=np.stack(irn),
                        gwphi=np.stack(gwphi), gwid=np.asarray(g.gwid), rind=rind, ia=ia, ig=ig,
                        gwind=g.get_gwrho_param_indices(), param_names=np.array(names))
    print("red likelihood:", out)


def pta_run(ref, out, kind, niter, n_psr=None):
    """Configs 4a/4b: PTABlockGibbs CURN (+ per-pulsar red free spectrum, conditional)."""
    pta = synthetic.array_pta(kind=kind, n_psr=n_psr, seed=0)
    np.random.seed(5)
    g = _quiet(ref.PTABlockGibbs, pta, hypersample="conditional",
               redsample="conditional" if kind == "curn_red" else "mh")
    x0 = np.concatenate([p.sample().flatten() for p in g.params])
    TNT, d, Ts = [], [], []
    N = pta.get_ndiag({})
    R = pta.get_residuals()
    for i, T in enumerate(pta.get_basis()):
        TNT.append(T.T @ (T / N[i][:, None]))
        d.append(T.T @ (R[i] / N[i]))
    m = np.array([t.shape[0] for t in TNT])
    off = np.concatenate([[0], np.cumsum(m)])
    # per-sweep record of every pulsar's b, before the sweep's update
    bhist = []
    with tempfile.TemporaryDirectory() as dd, Capture() as cap:
        np.random.seed(6)
        # run the reference loop one sweep at a time, recording b before each sweep
        g.chain = None
        chain = []
        xnew = x0
        for ii in range(niter):
            bhist.append(np.concatenate(g._b))
            # replicate sample()'s body exactly by calling sample with niter=ii+1 is
            # too slow; instead use the reference's own methods in sample()'s order
            chain.append(xnew.copy())
            if ii == 0:
                g._b = g.update_b(x0)
            g.TNT, g.d = [], []
            if g.get_hyper_param_indices().size != 0 and g.redsample == "conditional":
                xnew = g.update_hyper_params(xnew)
            xnew = g.update_rho_params(xnew)
            if np.all(xnew != chain[ii][-1]):
                g._b = g.update_b(xnew)
        _ = dd
    z = np.concatenate([a for a in cap.take("randn")])
    U = np.concatenate([a for a in cap.take("uniform")])
    np.savez_compressed(out, TNT=np.concatenate([t.ravel() for t in TNT]),
                        d=np.concatenate(d), m=m, off=off,
                        gwid=np.stack([np.asarray(gw) for gw in g.gwid]),
                        rhomin_gw=g.rhomin_gw, rhomax_gw=g.rhomax_gw,
                        rhomin_red=g.rhomin_red, rhomax_red=g.rhomax_red,
                        x0=x0, chain=np.stack(chain), bhist=np.stack(bhist),
                        b_final=np.concatenate(g._b), z=z, U=U,
                        rind=g.get_rho_param_indices(), hind=g.get_hyper_param_indices(),
                        param_names=np.array(g.param_names), pulsars=np.array(pta.pulsars))
    print("pta:", kind, out, z.shape, U.shape)


def pta_sample_check(ref, out, niter=101, n_psr=4):
    """PTABlockGibbs.sample itself (not our re-driven loop) on a small array: pins the loop order."""
    pta = synthetic.array_pta(kind="curn_red", n_psr=n_psr, seed=1)
    np.random.seed(7)
    g = _quiet(ref.PTABlockGibbs, pta, hypersample="conditional", redsample="conditional")
    x0 = np.concatenate([p.sample().flatten() for p in g.params])
    with tempfile.TemporaryDirectory() as d, Capture() as cap:
        np.random.seed(8)
        _quiet(g.sample, x0, outdir=d, niter=niter)
        saved = np.loadtxt(os.path.join(d, "chain.txt"))
    np.savez_compressed(out, x0=x0, chain=g.chain, saved_rows=saved.shape[0],
                        z=np.concatenate(cap.take("randn")), U=np.concatenate(cap.take("uniform")),
                        n_psr=n_psr)
    print("pta sample:", out, g.chain.shape, saved.shape)


def pta_long(ref, out, kind, niter=20000, seed=21, red_psr=(0,)):
    """Long PTABlockGibbs.sample chain on the 45-pulsar array (configs[3], north_star's target
    config) for the per-bin KS comparison of the device's CURN / CURN + red posteriors: the
    reference's own sample loop (pta_gibbs.py:631-713), single-threaded BLAS, seeded; keeps the
    common gw log10 rho columns (and the red bins of the pulsars in ``red_psr``) as float32."""
    pta = synthetic.array_pta(kind=kind, seed=0)
    np.random.seed(seed)
    g = _quiet(ref.PTABlockGibbs, pta, hypersample="conditional",
               redsample="conditional" if kind == "curn_red" else "mh")
    x0 = np.concatenate([p.sample().flatten() for p in g.params])
    with tempfile.TemporaryDirectory() as d:
        np.random.seed(seed + 1)
        _quiet(g.sample, x0, outdir=d, niter=niter)
    names = list(g.param_names)
    keep = [i for i, n in enumerate(names) if "gw" in n and "rho" in n]
    if kind == "curn_red":
        for p in red_psr:
            keep += [i for i, n in enumerate(names) if n.startswith(pta.pulsars[p] + "_") and "rho" in n]
    np.savez_compressed(out, chain=g.chain[:, keep].astype(np.float32), cols=np.array(keep),
                        names=np.array([names[i] for i in keep]), niter=niter, x0=x0, kind=kind)
    print("pta long:", kind, out, g.chain.shape)


def pta_hyper_mh(ref, out, kind="curn_plred", niter=8, warm=100, acl=20, n_psr=None, nlike=4):
    """PTABlockGibbs with the reference's DEFAULT redsample='mh' (pta_gibbs.py:278-340): per-pulsar
    red-noise hyper-parameters by single-parameter Metropolis on the summed marginalised likelihood
    get_lnlikelihood (:577-621), inside sample()'s order (:664-704), driven with the reference's own
    methods as pta_run does.  Sweep 0's warm-up branch (iters=100, :283-315) ends in np.cov /
    np.linalg.svd / acor of short_chain[100:], which is EMPTY for iters=100: numpy's SVD of the NaN
    covariance raises LinAlgError, so the reference cannot pass sweep 0 on its own default path
    (acor is absent here besides).  Its 100 MH steps are pinned through the steady-state branch
    (iters=None) with aclength_hyper = warm -- the same loop body, draws and acceptance -- and
    aclength_hyper = acl afterwards.  Every draw is captured (choice of scale, choice of parameter,
    randn jump, rand acceptance; CURN uniforms; b normals), plus x after each hyper block and the
    reference's get_lnlikelihood at a few states."""
    pta = synthetic.array_pta(kind=kind, n_psr=n_psr, seed=0)
    N = pta.get_ndiag({})
    R = pta.get_residuals()
    TNT, d = [], []
    for i, T in enumerate(pta.get_basis()):          # as update_b computes them (pta_gibbs.py:523-526)
        TNT.append(T.T @ (T / N[i][:, None]))
        d.append(T.T @ (R[i] / N[i]))
    np.random.seed(15)
    g = _quiet(ref.PTABlockGibbs, pta, hypersample="conditional", redsample="mh")
    x0 = np.concatenate([p.sample().flatten() for p in g.params])
    hind = g.get_hyper_param_indices()
    names = list(g.param_names)
    chain, hyper_in, hyper_out, bhist = [], [], [], []
    xnew = x0.copy()
    with Capture() as cap:
        np.random.seed(16)
        for ii in range(niter):
            chain.append(xnew.copy())
            bhist.append(np.concatenate(g._b))
            if ii == 0:
                g._b = g.update_b(x0)
            g.TNT, g.d = [], []
            g.aclength_hyper = warm if ii == 0 else acl
            hyper_in.append(xnew.copy())
            xnew = g.update_hyper_params(xnew, iters=None)
            hyper_out.append(xnew.copy())
            xnew = g.update_rho_params(xnew)
            if np.all(xnew != chain[ii][-1]):
                g._b = g.update_b(xnew)
    log = cap.log
    kinds = np.array([k for k, _ in log])
    vals = [v for _, v in log]
    # the reference's summed marginalised likelihood at a few states (no draws consumed)
    lstates = [hyper_in[0], hyper_out[0]] + hyper_out[1:nlike - 1]
    lnl = []
    for xs in lstates:
        g.TNT, g.d = [], []
        lnl.append(g.get_lnlikelihood(xs))
    np.savez_compressed(out, x0=x0, chain=np.stack(chain), bhist=np.stack(bhist), b_final=np.concatenate(g._b),
                        x_final=xnew, TNT=np.concatenate([t.ravel() for t in TNT]), d=np.concatenate(d),
                        off=np.concatenate([[0], np.cumsum([len(v) for v in d])]), n_psr=len(pta.pulsars),
                        hyper_in=np.stack(hyper_in), hyper_out=np.stack(hyper_out), kinds=kinds,
                        vals=np.concatenate([np.atleast_1d(v).ravel() for v in vals]),
                        lens=np.array([np.atleast_1d(v).size for v in vals]),
                        warm=warm, aclength=acl, hind=hind, rind=g.get_rho_param_indices(),
                        gwid=np.stack([np.asarray(gw) for gw in g.gwid]), m=np.array([len(b) for b in g._b]),
                        rhomin_gw=g.rhomin_gw, rhomax_gw=g.rhomax_gw, lnl_states=np.stack(lstates),
                        lnl=np.array(lnl), param_names=np.array(names), kind=kind,
                        pmin=np.array([p.pmin for p in g.params for _ in range(p.size or 1)]),
                        pmax=np.array([p.pmax for p in g.params for _ in range(p.size or 1)]))
    print("pta hyper mh:", kind, out, len(log), "accepted moves:",
          int(sum(np.sum(a != b) for a, b in zip(hyper_in, hyper_out))))


def pta_long_plred(ref, out, niter=40000, seed=31, n_psr=6, warm=100, acl=20, thin=10):
    """Long chain of the reference's DEFAULT PTA model (redsample='mh', power-law red noise per
    pulsar + CURN free spectrum) for the KS comparison of the device's curn_plred posteriors.
    sample() itself cannot pass sweep 0 on this path (its iters=100 warm-up ends in an SVD of the
    empty short_chain[100:] covariance, see pta_hyper_mh), so the reference's own methods are
    driven in sample()'s order (pta_gibbs.py:664-704) with sweep 0's 100 warm-up steps run through
    the steady-state branch (aclength_hyper = warm) and aclength_hyper = acl afterwards -- the
    patch pta_hyper_mh pins draw for draw.  Seeded, single-threaded BLAS; keeps the gw log10 rho
    and the red (log10_A, gamma) columns as float32, every ``thin``-th sweep."""
    pta = synthetic.array_pta(kind="curn_plred", n_psr=n_psr, seed=0)
    np.random.seed(seed)
    g = _quiet(ref.PTABlockGibbs, pta, hypersample="conditional", redsample="mh")
    x0 = np.concatenate([p.sample().flatten() for p in g.params])
    names = list(g.param_names)
    chain = np.empty((niter, len(x0)))
    xnew = x0.copy()
    np.random.seed(seed + 1)
    for ii in range(niter):
        chain[ii] = xnew
        if ii == 0:
            g._b = g.update_b(x0)
        g.TNT, g.d = [], []
        g.aclength_hyper = warm if ii == 0 else acl
        xnew = g.update_hyper_params(xnew, iters=None)
        xnew = g.update_rho_params(xnew)
        if np.all(xnew != chain[ii][-1]):
            g._b = g.update_b(xnew)
        if ii % 1000 == 0 or (n_psr > 6 and ii % 100 == 0):
            print("pta long plred", seed, ii, time.strftime("%H:%M:%S"), flush=True)
    keep = [i for i, n in enumerate(names) if ("gw" in n and "rho" in n) or "red_noise" in n]
    np.savez_compressed(out, chain=chain[::thin, keep].astype(np.float32), cols=np.array(keep),
                        names=np.array([names[i] for i in keep]), niter=niter, thin=thin, x0=x0,
                        kind="curn_plred", n_psr=n_psr, seed=seed, warm=warm, aclength=acl)
    print("pta long plred:", out, chain.shape)


def likelihoods(ref, out):
    """White-noise and fully-marginalised likelihoods (pulsar_gibbs.py:523-546, 569-610)."""
    pta = synthetic.single_pulsar_pta("J1713+0747", seed=0, efac_vary=True, n_backends=3)
    np.random.seed(9)
    g = _quiet(ref.PulsarBlockGibbs, pta)
    rs = np.random.RandomState(10)
    xs, white, marg, bs = [], [], [], []
    for _ in range(8):
        x = np.concatenate([p.sample().flatten() for p in g.params])
        b = rs.standard_normal(len(g._b)) * 1e-7
        g._b = b
        g.TNT = g.d = None
        xs.append(x), bs.append(b)
        white.append(g.get_lnlikelihood_white(x))
        g.TNT = g.d = None
        marg.append(g.get_lnlikelihood_fullmarg(x))
    sig = pta.models[0].white[0]
    np.savez_compressed(out, x=np.stack(xs), b=np.stack(bs), white=np.array(white),
                        marg=np.array(marg), T=pta.get_basis()[0], r=pta.get_residuals()[0],
                        sigma=sig.sigma, backends=sig.backends,
                        param_names=np.array(g.param_names))
    print("likelihoods:", out)


def white_mh(ref, out, nsweep=6, acl=40):
    """White-noise Metropolis block (pulsar_gibbs.py:332-406, steady-state branch)
    inside the sample loop order (:656-698), driven with the reference's own methods.
    The warm-up branch (iters=1000) needs `acor` (absent here), so aclength_white is
    set directly; every MH draw (choice of scale, choice of parameter, randn jump,
    rand acceptance) is captured."""
    pta = synthetic.single_pulsar_pta("J1713+0747", seed=0, efac_vary=True, n_backends=3)
    np.random.seed(13)
    g = _quiet(ref.PulsarBlockGibbs, pta)
    x0 = np.concatenate([p.sample().flatten() for p in g.params])
    names = list(g.param_names)
    wind = g.get_efacequad_indices()
    g.aclength_white = acl
    chain, bhist, white_in, white_out = [], [], [], []
    xnew = x0.copy()
    with Capture() as cap:
        np.random.seed(14)
        for ii in range(nsweep):
            chain.append(xnew.copy())
            bhist.append(g._b.copy())
            if ii == 0:
                g._b = g.update_b(x0)
            g.TNT = g.d = None
            white_in.append(xnew.copy())
            xnew = g.update_white_params(xnew, iters=None)
            white_out.append(xnew.copy())
            xnew = g.update_gwrho_params(xnew)
            if np.all(xnew != chain[ii][-1]):
                g._b = g.update_b(xnew)
    log = cap.log
    kinds = np.array([k for k, _ in log])
    vals = [v for _, v in log]
    sig = pta.models[0].white[0]
    np.savez_compressed(out, x0=x0, chain=np.stack(chain), bhist=np.stack(bhist), b_final=g._b,
                        white_in=np.stack(white_in), white_out=np.stack(white_out),
                        kinds=kinds, vals=np.concatenate([np.atleast_1d(v).ravel() for v in vals]),
                        lens=np.array([np.atleast_1d(v).size for v in vals]),
                        T=pta.get_basis()[0], r=pta.get_residuals()[0], sigma=sig.sigma,
                        backends=sig.backends, wind=wind, aclength=acl, gwid=np.asarray(g.gwid),
                        rhomin=g.rhomin, rhomax=g.rhomax, param_names=np.array(names),
                        pmin=np.array([p.pmin for p in g.params for _ in range(p.size or 1)]),
                        pmax=np.array([p.pmax for p in g.params for _ in range(p.size or 1)]))
    print("white:", out, len(log))


def ecorr_mh(ref, out, nsweep=6, acl=30, nlike=8):
    """Basis-ECORR Metropolis block: PulsarBlockGibbs.update_ecorr_params
    (pulsar_gibbs.py:409-486, steady-state branch) whose self.get_lnlikelihood the .py never
    defines -- bound here to the reference's own get_lnlikelihood_fullmarg (:569-610), the
    same code as the notebook's get_lnlikelihood (pta_gibbs_freespec.ipynb, cell 2) -- inside
    the notebook's sweep order (ECORR block, rho|b, gated b).  aclength_ecorr is set directly
    (its warm-up needs `acor`, absent).  Also the marginalised likelihood at prior draws."""
    pta = synthetic.ecorr_pulsar_pta("J1713+0747", seed=0)
    np.random.seed(21)
    g = _quiet(ref.PulsarBlockGibbs, pta)
    g.get_lnlikelihood = g.get_lnlikelihood_fullmarg
    x0 = np.concatenate([p.sample().flatten() for p in g.params])
    eind = g.get_ecorr_indices()
    g.aclength_ecorr = acl
    rs = np.random.RandomState(22)
    xl, ll = [], []
    for i in range(nlike):
        x = np.concatenate([p.sample().flatten() for p in g.params])
        if i == nlike - 1:
            x[eind] = [p.pmin for p in g.params if "ecorr" in p.name]   # prior edge
        g.TNT = g.d = None
        xl.append(x), ll.append(g.get_lnlikelihood_fullmarg(x))
    chain, bhist, e_in, e_out = [], [], [], []
    xnew = x0.copy()
    with Capture() as cap:
        np.random.seed(23)
        for ii in range(nsweep):
            chain.append(xnew.copy())
            bhist.append(g._b.copy())
            if ii == 0:
                g._b = g.update_b(x0)
            g.TNT = g.d = None
            e_in.append(xnew.copy())
            xnew = g.update_ecorr_params(xnew, iters=None)
            e_out.append(xnew.copy())
            xnew = g.update_gwrho_params(xnew)
            if np.all(xnew != chain[ii][-1]):
                g._b = g.update_b(xnew)
    log = cap.log
    sig = pta.signals["J1713+0747_basis_ecorr"]
    np.savez_compressed(out, x0=x0, chain=np.stack(chain), bhist=np.stack(bhist), b_final=g._b,
                        e_in=np.stack(e_in), e_out=np.stack(e_out),
                        kinds=np.array([k for k, _ in log]),
                        vals=np.concatenate([np.atleast_1d(v).ravel() for _, v in log]),
                        lens=np.array([np.atleast_1d(v).size for _, v in log]),
                        T=pta.get_basis()[0], r=pta.get_residuals()[0], Nvec=pta.get_ndiag()[0],
                        epoch_backend=sig.epoch_backend, eind=eind, ecid=np.asarray(g.ecid),
                        aclength=acl, gwid=np.asarray(g.gwid), rhomin=g.rhomin, rhomax=g.rhomax,
                        ecorrmin=g.ecorrmin, ecorrmax=g.ecorrmax, param_names=np.array(g.param_names),
                        x_like=np.stack(xl), lnlike=np.array(ll),
                        pmin=np.array([p.pmin for p in g.params for _ in range(p.size or 1)]),
                        pmax=np.array([p.pmax for p in g.params for _ in range(p.size or 1)]))
    print("ecorr:", out, len(log))


def ecorr_long(ref, out, niter=6000, thin=5, acl=10):
    """Long reference run of the ECORR sweep (ecorr_mh's loop, no draw capture) for the
    posterior comparison: x thinned by `thin`."""
    pta = synthetic.ecorr_pulsar_pta("J1713+0747", seed=0)
    np.random.seed(31)
    g = _quiet(ref.PulsarBlockGibbs, pta)
    g.get_lnlikelihood = g.get_lnlikelihood_fullmarg
    g.aclength_ecorr = acl
    x0 = np.concatenate([p.sample().flatten() for p in g.params])
    xnew = x0.copy()
    rows = []
    for ii in range(niter):
        if ii % thin == 0:
            rows.append(xnew.copy())
        xold_last = xnew[-1]
        if ii == 0:
            g._b = g.update_b(x0)
        g.TNT = g.d = None
        xnew = g.update_ecorr_params(xnew, iters=None)
        xnew = g.update_gwrho_params(xnew)
        if np.all(xnew != xold_last):
            g._b = g.update_b(xnew)
    np.savez_compressed(out, x0=x0, chain=np.stack(rows), thin=thin, aclength=acl)
    print("ecorr long:", out, len(rows))


def ecorr_white_mh(ref, out, nsweep=5, acl_w=12, acl_e=12, nlike=6):
    """White-noise + basis-ECORR blocks together (the notebook J1713 configuration,
    white_vary=True): per sweep (notebook sample order) record, [first b], TNT reset,
    update_white_params (:373-404, steady state), update_ecorr_params (:456-484, its
    get_lnlikelihood = get_lnlikelihood_fullmarg), rho|b, gated b; every draw captured.
    Also the marginalised likelihood at prior draws of all parameters."""
    pta = synthetic.ecorr_pulsar_pta("J1713+0747", seed=0, white_vary=True)
    np.random.seed(41)
    g = _quiet(ref.PulsarBlockGibbs, pta)
    g.get_lnlikelihood = g.get_lnlikelihood_fullmarg
    x0 = np.concatenate([p.sample().flatten() for p in g.params])
    wind, eind = g.get_efacequad_indices(), g.get_ecorr_indices()
    x0[wind] = [1.0 if "efac" in n else -7.0 for n in np.array(g.param_names)[wind]]
    g.aclength_white, g.aclength_ecorr = acl_w, acl_e
    xl, ll = [], []
    for _ in range(nlike):
        x = np.concatenate([p.sample().flatten() for p in g.params])
        g.TNT = g.d = None
        xl.append(x), ll.append(g.get_lnlikelihood_fullmarg(x))
    chain, bhist, w_in, w_out, e_out = [], [], [], [], []
    xnew = x0.copy()
    with Capture() as cap:
        np.random.seed(43)
        for ii in range(nsweep):
            chain.append(xnew.copy())
            bhist.append(g._b.copy())
            if ii == 0:
                g._b = g.update_b(x0)
            g.TNT = g.d = None
            w_in.append(xnew.copy())
            xnew = g.update_white_params(xnew, iters=None)
            w_out.append(xnew.copy())
            xnew = g.update_ecorr_params(xnew, iters=None)
            e_out.append(xnew.copy())
            xnew = g.update_gwrho_params(xnew)
            if np.all(xnew != chain[ii][-1]):
                g._b = g.update_b(xnew)
    log = cap.log
    sig = pta.signals["J1713+0747_basis_ecorr"]
    wn = pta.models[0].white[0]
    np.savez_compressed(out, x0=x0, chain=np.stack(chain), bhist=np.stack(bhist), b_final=g._b,
                        w_in=np.stack(w_in), w_out=np.stack(w_out), e_out=np.stack(e_out),
                        kinds=np.array([k for k, _ in log]),
                        vals=np.concatenate([np.atleast_1d(v).ravel() for _, v in log]),
                        lens=np.array([np.atleast_1d(v).size for _, v in log]),
                        T=pta.get_basis()[0], r=pta.get_residuals()[0], sigma=wn.sigma, backends=wn.backends,
                        epoch_backend=sig.epoch_backend, eind=eind, wind=wind, ecid=np.asarray(g.ecid),
                        aclength_white=acl_w, aclength_ecorr=acl_e, gwid=np.asarray(g.gwid),
                        rhomin=g.rhomin, rhomax=g.rhomax, param_names=np.array(g.param_names),
                        x_like=np.stack(xl), lnlike=np.array(ll),
                        pmin=np.array([p.pmin for p in g.params for _ in range(p.size or 1)]),
                        pmax=np.array([p.pmax for p in g.params for _ in range(p.size or 1)]))
    print("ecorr+white:", out, len(log))


def indep_runs(ref, out, niter=60, picks=("B1937+21", "J1455-3330", "J1909-3744")):
    """BASELINE configs[2]: 45 independent pulsars, each its own PulsarBlockGibbs
    (pulsar_gibbs.py:620-710) on its own free spectrum.  The reference has no array
    sampler, so a user runs PulsarBlockGibbs per pulsar; this fixture runs the reference
    on three of them (the smallest, a middle and the largest m: 68, 74, 77) with every
    draw captured."""
    pta = synthetic.array_pta(kind="indep", seed=0)
    ptas = synthetic.pulsar_ptas(pta)
    names = [p.pulsars[0] for p in ptas]
    rec = dict(pulsars=np.array(names), picks=np.array([names.index(n) for n in picks]))
    for k, n in enumerate(picks):
        pp = ptas[names.index(n)]
        np.random.seed(100 + k)
        g = _quiet(ref.PulsarBlockGibbs, pp)
        x0 = np.concatenate([p.sample().flatten() for p in g.params])
        with tempfile.TemporaryDirectory() as d, Capture() as cap:
            np.random.seed(200 + k)
            _quiet(g.sample, x0, outdir=d, niter=niter)
        rec.update({f"p{k}_T": pp.get_basis()[0], f"p{k}_Nvec": pp.get_ndiag({})[0],
                    f"p{k}_r": pp.get_residuals()[0], f"p{k}_x0": x0, f"p{k}_z": np.stack(cap.take("randn")),
                    f"p{k}_U": np.stack(cap.take("uniform")), f"p{k}_chain": g.chain,
                    f"p{k}_bchain": g.bchain, f"p{k}_b_final": g._b, f"p{k}_gwid": np.asarray(g.gwid),
                    f"p{k}_rhomin": g.rhomin, f"p{k}_rhomax": g.rhomax,
                    f"p{k}_param_names": np.array(g.param_names)})
    np.savez_compressed(out, niter=niter, **rec)
    print("indep:", out, [rec[f"p{k}_z"].shape for k in range(len(picks))])


def main(root):
    mods = load_reference(root)
    PB = mods["pulsar_gibbs"]
    PT = mods["pta_gibbs"]
    if "--only-indep" in sys.argv:
        indep_runs(PB, os.path.join(HERE, "indep_array.npz"))
        return
    if "--only-ecorr-white" in sys.argv:
        ecorr_white_mh(PB, os.path.join(HERE, "ecorr_white_j1713.npz"))
        return
    if "--only-ecorr" in sys.argv:
        ecorr_mh(PB, os.path.join(HERE, "ecorr_mh_j1713.npz"))
        if "--long" in sys.argv:
            ecorr_long(PB, os.path.join(HERE, "ecorr_long_j1713.npz"))
        return
    for kind in ("curn", "curn_red"):
        if f"--only-pta-long-{kind}" in sys.argv:
            pta_long(PT, os.path.join(HERE, f"pta_long_{kind}.npz"), kind)
            return
    if "--only-pta-long-plred" in sys.argv:
        # one seed per process: --seed=S --niter=N -> pta_long_curn_plred_s{S}.npz
        opt = dict(a[2:].split("=", 1) for a in sys.argv if a.startswith("--") and "=" in a)
        s = int(opt.get("seed", 31))
        n_psr = int(opt.get("npsr", 6))
        tag = f"pta_long_curn_plred_s{s}.npz" if n_psr == 6 else f"pta_long_curn_plred_p{n_psr}_s{s}.npz"
        pta_long_plred(PT, os.path.join(HERE, tag), niter=int(opt.get("niter", 40000)), seed=s, n_psr=n_psr,
                       thin=int(opt.get("thin", 10)))
        return
    if "--only-pta-mh" in sys.argv:
        pta_hyper_mh(PT, os.path.join(HERE, "pta_plred_mh.npz"), "curn_plred")
        pta_hyper_mh(PT, os.path.join(HERE, "pta_red_mh.npz"), "curn_red", n_psr=6, niter=6, acl=30)
        return
    if "--only-red" in sys.argv:
        red_likelihood(PB, os.path.join(HERE, "red_lnlike_j1713.npz"))
        return
    single_pulsar(PB, os.path.join(HERE, "single_j1713.npz"))
    single_pulsar_gumbel(PB, os.path.join(HERE, "gumbel_j1713.npz"))
    likelihoods(PB, os.path.join(HERE, "likelihoods_j1713.npz"))
    pta_run(PT, os.path.join(HERE, "pta_curn.npz"), "curn", niter=12)
    pta_run(PT, os.path.join(HERE, "pta_curn_red.npz"), "curn_red", niter=12)
    pta_sample_check(PT, os.path.join(HERE, "pta_sample_small.npz"))
    pta_hyper_mh(PT, os.path.join(HERE, "pta_plred_mh.npz"), "curn_plred")
    pta_hyper_mh(PT, os.path.join(HERE, "pta_red_mh.npz"), "curn_red", n_psr=6, niter=6, acl=30)
    white_mh(PB, os.path.join(HERE, "white_mh_j1713.npz"))
    red_likelihood(PB, os.path.join(HERE, "red_lnlike_j1713.npz"))
    ecorr_mh(PB, os.path.join(HERE, "ecorr_mh_j1713.npz"))
    ecorr_white_mh(PB, os.path.join(HERE, "ecorr_white_j1713.npz"))
    indep_runs(PB, os.path.join(HERE, "indep_array.npz"))
    if "--long" in sys.argv:
        single_pulsar_long(PB, os.path.join(HERE, "long_j1713.npz"))
        ecorr_long(PB, os.path.join(HERE, "ecorr_long_j1713.npz"))


if __name__ == "__main__":
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    main(args[0] if args else "/root/reference")
