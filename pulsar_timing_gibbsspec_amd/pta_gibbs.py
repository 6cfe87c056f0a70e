"""``PTABlockGibbs`` — drop-in for the reference's multi-pulsar sampler.

Mirrors ``/root/reference/pta_gibbs.py:14-713`` for the common free-spectrum
(CURN) model with optional per-pulsar red free spectra drawn conditionally
(``redsample='conditional'``): same constructor, parameter plumbing, prior
parsing, per-pulsar gwid discovery, ``update_b`` / ``update_rho_params`` /
``update_hyper_params`` / ``sample`` surface and ``chain.txt`` output.  All
arithmetic runs on the GPU (engine.PTAChains); chains are batched
(``nchains``), chain 0 is written in the reference layout.

Per-pulsar red noise: ``redsample='conditional'`` (free spectrum, grid-CDF draws) or the
reference's default ``redsample='mh'`` (power-law or free-spectrum red noise by the
single-parameter Metropolis block on the summed marginalised likelihood,
pta_gibbs.py:278-340; device kernels in ``pta_hyper``).

Outside the device hot path (raise NotImplementedError): the white-noise / ECORR Metropolis
blocks of the PTA class (single-pulsar code inside the array sampler, pta_gibbs.py:551-575)
and ``hypersample='mh'`` (dead code).
"""
from __future__ import annotations

import os
import sys
import time

import numpy as np
import torch

from . import _lib
from .engine import DeviceModel, PTAChains
from .plumbing import basis_layout, expand_names, last_match, matching_indices, power_bounds, vector_to_dict
from .pta_hyper import HYPER_WARMUP, HyperSpec, hyper_aclength
from .pulsar_gibbs import HOST_CHAIN, resolve_seed


class PTABlockGibbs(object):
    """Gibbs-based pulsar-timing periodogram analysis of a PTA on MI355X
    (van Haasteren & Vallisneri 2014)."""

    def __init__(self, pta, hypersample="conditional", redsample="mh", *, nchains=1, device=0,
                 seed=None, curn_mode="auto"):
        # the common draw (pta_gibbs.py:181-214): 'exact' = the product of per-pulsar pdfs;
        # 'sum' = the same law from the tau sums (no per-pulsar red noise only); 'auto' picks
        # 'sum' when the model has no per-pulsar red free spectrum
        if curn_mode not in ("auto", "exact", "sum"):
            raise ValueError("curn_mode must be 'auto', 'exact' or 'sum'")
        self.curn_mode = curn_mode
        self.pta = pta
        self.hypersample = hypersample
        self.redsample = redsample
        self.nchains = int(nchains)
        # the reference only warns here (pta_gibbs.py:62-66)
        if not any("basis_ecorr" in key for key in pta._signal_dict):
            print("ERROR: Gibbs outlier analysis must use basis_ecorr, not kernel ecorr")

        self._residuals = pta.get_residuals()
        T0 = pta.get_basis([p.sample() for p in pta.params])
        self._b = [np.zeros(T0[i].shape[1]) for i in range(len(pta.pulsars))]
        self.TNT = []
        self.d = []

        # prior bounds (pta_gibbs.py:83-94): the last 'gw'+'rho' parameter, then the last
        # 'red'+'rho' one -- which, as in the reference, stays the gw parameter when the
        # model has no red free spectrum
        pnames = [p.name for p in self.params]
        ind = last_match(pnames, lambda n: "rho" in n and "gw" in n)
        if ind is None:
            raise UnboundLocalError("no common 'gw' ... 'rho' parameter in the PTA")
        self.rhomin_gw, self.rhomax_gw = power_bounds(self.params[ind].params[0])
        red = last_match(pnames, lambda n: "rho" in n and "red" in n)
        self.rhomin_red, self.rhomax_red = power_bounds(self.params[ind if red is None else red].params[0])

        # per-pulsar gw columns, each pulsar's signals walked alone (pta_gibbs.py:96-109)
        self.gwid = [basis_layout(pta.signals, [k for k in pta.signals if pname in k])[0]
                     for pname in pta.pulsars]

        sigs = [pta.signals[k] for k in pta.signals]
        self.red_sig = [s for s in sigs if "red" in s.name]
        self.gw_sig = next((s for s in reversed(sigs) if "gw" in s.name), None)

        self.seed, self._key = resolve_seed(seed)
        self._device = device
        self._ctx = None
        self._device_model = None
        self._engine = None

    @property
    def ctx(self):
        if self._ctx is None:
            self._ctx = _lib.Context(self._device, seed=self._key)
        return self._ctx

    # ------------------------------------------------------------ plumbing
    @property
    def params(self):
        return list(self.pta.params)

    @property
    def param_names(self):
        return expand_names(self.params)

    def map_params(self, xs):
        return vector_to_dict(self.params, xs)

    def _indices(self, pred):
        return matching_indices(self.param_names, pred)

    def get_rho_param_indices(self):
        return self._indices(lambda par: "rho" in par and "gw" in par)

    def get_hyper_param_indices(self):
        return self._indices(lambda par: "red" in par and ("log10_A" in par or "gamma" in par or "rho" in par))

    def get_efacequad_indices(self):
        return self._indices(lambda par: "efac" in par or "equad" in par)

    def get_ecorr_indices(self):
        return self._indices(lambda par: "ecorr" in par)

    def get_lnprior(self, params):
        params = params if isinstance(params, dict) else self.map_params(params)
        return np.sum([p.get_logpdf(params=params) for p in self.params])

    # ------------------------------------------------------------ device state
    def _check_supported(self):
        if self.hypersample != "conditional":
            raise NotImplementedError("hypersample='mh' (Metropolis on rho) is outside the device hot path")
        if self.get_efacequad_indices().size or self.get_ecorr_indices().size:
            raise NotImplementedError("white-noise / ECORR Metropolis blocks are outside the device PTA path")
        hind = self.get_hyper_param_indices()
        if self.redsample not in ("conditional", "mh"):
            raise ValueError("redsample must be 'conditional' or 'mh'")
        if hind.size and self.redsample == "conditional" and \
                hind.size != len(self.pta.pulsars) * (len(self.gwid[0]) // 2):
            raise NotImplementedError("redsample='conditional' needs per-pulsar red free spectra on the gw basis")
        if hind.size and self.redsample == "mh":
            self._hyper_spec()          # raises for red models other than power law / free spectrum
        n_known = self.get_rho_param_indices().size + hind.size
        if n_known != len(self.param_names):
            raise NotImplementedError("parameters other than gw/red free-spectrum powers are not supported")

    def _model(self, xs):
        if self._device_model is not None:
            return self._device_model
        params = self.map_params(xs)
        T = self.pta.get_basis(params)
        N = self.pta.get_ndiag(params)
        ph = self.pta.get_phiinv(params, logdet=False)
        fixed = []
        for p in range(len(T)):
            mask = np.ones(T[p].shape[1], bool)
            mask[self.gwid[p]] = False
            fixed.append(ph[p][mask])
        self._device_model = DeviceModel(self.ctx, T, N, self._residuals, self.gwid, fixed)
        for p in range(len(T)):
            a, b = self._device_model.tnt_host(p)
            self.TNT.append(a)
            self.d.append(b)
        return self._device_model

    def _hyper_spec(self):
        """Device tables of the red hyper-parameters (redsample='mh'), built once."""
        if getattr(self, "_hspec", None) is None:
            n_f = len(self.gwid[0]) // 2
            x_ref = np.zeros(len(self.param_names))    # only each red signal's own parameters are probed
            self._hspec = HyperSpec(self.pta, self.params, self.red_sig, self.get_hyper_param_indices(), x_ref,
                                    n_f, self.ctx.device)
        return self._hspec

    def _new_engine(self, xs, chain_base=0):
        self._check_supported()
        model = self._model(xs)
        hind = self.get_hyper_param_indices()
        if hind.size and self.redsample == "mh":
            return PTAChains(model, len(self.param_names), self.get_rho_param_indices(), None,
                             (self.rhomin_gw, self.rhomax_gw), (self.rhomin_red, self.rhomax_red),
                             self.nchains, np.asarray(xs, float), chain_base=chain_base, curn_mode="exact",
                             hyper=self._hyper_spec(), hyper_acl=getattr(self, "aclength_hyper", None),
                             hyper_warmup=HYPER_WARMUP)
        red_col = hind.reshape(len(self.pta.pulsars), -1) if hind.size else None
        mode = self.curn_mode
        if mode == "auto":
            # 'sum' needs every tau inside its fixed-point window [rhomin_gw 2^-64, rhomin_gw 2^80):
            # a prior wider than ~2^80 / 1e4 (tau reaches a few x 1e3 rhomax) falls back to 'exact'
            wide = self.rhomax_gw / self.rhomin_gw > 2.0 ** 80 / 1e4
            mode = "exact" if (red_col is not None or wide) else "sum"
        return PTAChains(model, len(self.param_names), self.get_rho_param_indices(), red_col,
                         (self.rhomin_gw, self.rhomax_gw), (self.rhomin_red, self.rhomax_red),
                         self.nchains, np.asarray(xs, float), chain_base=chain_base, curn_mode=mode)

    # ------------------------------------------------------------ conditionals (single-call API)
    def _engine_at(self, xs):
        """The single-call API's own engine: chain ids from HOST_CHAIN, so its Philox draws
        never repeat those of a sample() run (chains 0 .. nchains - 1)."""
        eng = self._api_engine if getattr(self, "_api_engine", None) is not None else \
            self._new_engine(xs, chain_base=HOST_CHAIN)
        self._api_engine = eng
        eng.x.copy_(torch.as_tensor(np.asarray(xs, float), device=self.ctx.device).expand_as(eng.x))
        b = np.zeros((len(self._b), eng.model.ldb))
        for p, bb in enumerate(self._b):
            b[p, :bb.size] = bb
        eng.b.copy_(torch.as_tensor(np.repeat(b, eng.C, axis=0), device=self.ctx.device))
        # the per-pulsar red phi (irn) at xs: the gate's phiinv and the common draw read it
        # (power-law red noise or a red free spectrum; without red noise irn is None)
        eng._update_irn()
        return eng

    def update_b(self, xs):
        """b | rho for every pulsar (pta_gibbs.py:512-548), on the GPU."""
        eng = self._engine_at(xs)
        eng._gate_phiinv(with_gate=False)
        eng._bdraw(None, _lib.EV_USER, None)
        eng.it += 1
        b = eng.b.cpu().numpy()
        return [b[p * eng.C, :eng.model.m[p]] for p in range(eng.P)]

    def update_rho_params(self, xs):
        """Common free spectrum | b (pta_gibbs.py:181-214), on the GPU."""
        eng = self._engine_at(xs)
        lib, h, m = self.ctx.lib, self.ctx.handle, eng.model
        _lib.check(lib.gs_tau(h, eng.P, eng.C, m.NF, m.ldb, _lib.ptr(m.fidx), _lib.ptr(eng.b), 0,
                              _lib.ptr(eng.tau)), "gs_tau")
        _lib.check(lib.gs_rho_curn(h, eng.P, eng.C, eng.n_f, _lib.ptr(eng.tau), _lib.ptr(eng.irn),
                                   eng.ngrid, _lib.ptr(eng.grid_gw), None, eng.it, eng.chain_base, _lib.ptr(eng.x),
                                   eng.n_param, _lib.ptr(eng.gw_col), None), "gs_rho_curn")
        eng.it += 1
        return eng.x[0].cpu().numpy()

    def get_lnlikelihood(self, xs):
        """Summed marginalised likelihood of every pulsar (pta_gibbs.py:577-621) at xs, on the
        GPU: -1/2 (log det N + r^T N^-1 r) + 1/2 (d^T Sigma^-1 d - log det Sigma - log det phi) per
        pulsar; -inf if a Sigma is not positive definite."""
        eng = self._engine_at(xs)
        ph = torch.empty(eng.P * eng.C, eng.model.NF, dtype=torch.float64, device=self.ctx.device)
        gate = torch.empty(eng.C, dtype=torch.int32, device=self.ctx.device)
        if eng.phi_shared:
            check_phi = eng.phiinv_F
            eng._gate_phiinv(with_gate=False)
            ph.copy_(check_phi[:eng.C].repeat(eng.P, 1))
        else:
            eng._gate_phiinv(with_gate=False, out=ph, gate=gate)
        lnl, info = eng.model.lnlike_marg(ph, eng.C)
        lnl = lnl.view(eng.P, eng.C)[:, 0].cpu().numpy()
        if info.view(eng.P, eng.C)[:, 0].any():
            return -np.inf
        return float(np.sum(lnl))

    def update_hyper_params(self, xs, iters=None):
        """Per-pulsar red noise (pta_gibbs.py:246-342), on the GPU: redsample='conditional' ->
        red free spectra | b, phi_gw by the grid CDF; redsample='mh' -> ``iters`` (warm-up: sets
        cov_hyper, sigma_hyper, svd_hyper and aclength_hyper from the proposal chain,
        :309-315) or ``aclength_hyper`` Metropolis steps on the marginalised likelihood."""
        if self.redsample == "mh":
            eng = self._engine_at(xs)
            if eng.hyper is None:
                return np.asarray(xs, float).copy()
            if iters is not None and int(iters) <= 0:
                raise ValueError(f"iters must be positive (got {iters})")
            n = int(iters) if iters is not None else int(self.aclength_hyper)
            q_rec = torch.empty(n, eng.C, 3, dtype=torch.float64, device=self.ctx.device) \
                if iters is not None else None
            eng.hyper_block(n, q_rec=q_rec)
            eng.it += 1
            if iters is not None:
                sc = self._hspec.short_chain(np.asarray(xs, float), q_rec[:, 0].cpu().numpy())
                body = sc[100:] if sc.shape[0] > 100 else sc
                self.cov_hyper = np.atleast_2d(np.cov(body, rowvar=False))
                self.sigma_hyper = np.diag(self.cov_hyper) ** 0.5
                self.svd_hyper = np.linalg.svd(self.cov_hyper)
                self.aclength_hyper = hyper_aclength(sc)
            return eng.x[0].cpu().numpy()
        eng = self._engine_at(xs)
        if not eng.red:
            return np.asarray(xs, float).copy()
        lib, h, m = self.ctx.lib, self.ctx.handle, eng.model
        _lib.check(lib.gs_tau(h, eng.P, eng.C, m.NF, m.ldb, _lib.ptr(m.fidx), _lib.ptr(eng.b), 0,
                              _lib.ptr(eng.tau)), "gs_tau")
        _lib.check(lib.gs_phi_from_x(h, eng.C, eng.n_f, _lib.ptr(eng.x), eng.n_param, _lib.ptr(eng.gw_col),
                                     _lib.ptr(eng.gwphi)), "gs_phi_from_x")
        _lib.check(lib.gs_rho_red(h, eng.P, eng.C, eng.n_f, _lib.ptr(eng.tau), _lib.ptr(eng.gwphi), eng.ngrid,
                                  _lib.ptr(eng.grid_red), None, eng.it, eng.chain_base, _lib.ptr(eng.x), eng.n_param,
                                  _lib.ptr(eng.red_col), None), "gs_rho_red")
        eng.it += 1
        return eng.x[0].cpu().numpy()

    # ------------------------------------------------------------ resume state
    @staticmethod
    def _save_state(outdir, rows, eng):
        """gibbs_state.npz next to chain.txt: every chain's x and every (pulsar, chain)
        b BEFORE sweep ``rows`` -- what resume needs to continue bit for bit (the reference
        keeps no b on disk, pta_gibbs.py:707-712)."""
        extra = {} if eng.hyper is None else {"aclength_hyper": eng.hyper_acl}
        np.savez(f"{outdir}/gibbs_state.npz", rows=rows, x=eng.x.cpu().numpy(), b=eng.b.cpu().numpy(), **extra)

    def _load_state(self, outdir, rows, npar):
        f = f"{outdir}/gibbs_state.npz"
        if not os.path.exists(f):
            return None
        st = np.load(f, allow_pickle=False)
        if int(st["rows"]) != rows or st["x"].shape != (self.nchains, npar):
            return None
        return st

    # ------------------------------------------------------------ loop
    def sample(self, xs, outdir="./", niter=10000, resume=False, save_every=100, *, flush_final=False):
        """PTABlockGibbs.sample (pta_gibbs.py:631-713): chain row ii = state before sweep ii;
        chain.txt (chain 0) rewritten with rows [:ii+1] at ii % 100 == 0, ii > 0;
        with nchains > 1 also chains.npy (leading chain axis).  flush_final=True also
        writes the rows after the last multiple of save_every (the reference
        drops them, Appendix A.8)."""
        print(f"Creating chain directory: {outdir}")
        os.makedirs(outdir, exist_ok=True)
        self._check_supported()
        nc = self.nchains
        npar = len(xs)
        self.chain = np.zeros((niter, npar))
        self.chains = np.zeros((nc, niter, npar)) if nc > 1 else None
        self.iter = 0
        start = 0
        x0 = np.asarray(xs, float)
        state = None
        if resume and os.path.exists(f"{outdir}/chain.txt"):
            print("Resuming from previous run...")
            prev = np.atleast_2d(np.loadtxt(f"{outdir}/chain.txt"))
            start = prev.shape[0]
            self.chain[:start] = prev
            x0 = prev[-1]
            state = self._load_state(outdir, start, npar)
            if nc > 1 and os.path.exists(f"{outdir}/chains.npy"):
                prevc = np.load(f"{outdir}/chains.npy")
                if prevc.shape[0] == nc and prevc.shape[1] >= start:
                    self.chains[:, :start] = prevc[:, :start]
        eng = self._new_engine(x0)
        self._engine = eng
        dev = self.ctx.device
        buf = torch.empty(save_every + 1, nc, npar, dtype=torch.float64, device=dev)
        tstart = time.time()
        ii = start
        seen_fail = 0
        if start > 0:
            eng.it = start
            if eng.hyper is not None and eng.hyper_acl is None:
                if state is not None and "aclength_hyper" in state.files:
                    eng.hyper_acl = int(state["aclength_hyper"])
                else:
                    raise NotImplementedError("resuming a redsample='mh' run needs aclength_hyper (set the "
                                              "attribute, or keep gibbs_state.npz)")
            if state is not None:
                # the device state saved with these rows (gibbs_state.npz): the run continues
                # exactly where the uninterrupted one would be
                eng.x.copy_(torch.as_tensor(state["x"], device=dev))
                eng.b.copy_(torch.as_tensor(state["b"], device=dev))
            else:
                # only chain.txt (e.g. written by the reference): as pta_gibbs.py:642-661,
                # restart from the last row, which the next sweep records again -- but draw
                # b | x first (the reference keeps b = 0 there, which makes tau = 0 and the
                # grid CDF 0/0)
                eng.redraw_b = True
        while ii < niter:
            nxt = min(niter, (ii // save_every + 1) * save_every + 1)
            for j in range(nxt - ii):
                eng.sweep(x_rec=buf[j])
            rows = buf[:nxt - ii].cpu().numpy()
            eng.check_fx()                             # curn_mode='sum': tau inside the fixed-point window
            nfail = int(eng.fail_count.sum())          # failed (non-PD) b draws, b kept
            if nfail > seen_fail:
                print(f"WARNING: sweeps {ii}..{nxt - 1}: {nfail - seen_fail} b draws hit a non-positive-definite "
                      "Sigma; those systems KEEP their previous b -- unlike the reference, whose LinAlgError "
                      "branch (pta_gibbs.py:539-544) redraws b from a QR/SVD of Sigma with the wrong covariance "
                      "(SURVEY Appendix A.7)")
                seen_fail = nfail
            self.chain[ii:nxt] = rows[:, 0]
            if nc > 1:
                self.chains[:, ii:nxt] = np.moveaxis(rows, 1, 0)
            ii = nxt
            self.iter = ii - 1
            last = ii - 1
            if last % save_every == 0 and last > 0:
                sys.stdout.write("\r")
                sys.stdout.write("Finished %g percent in %g seconds." % (last / niter * 100, time.time() - tstart))
                sys.stdout.flush()
                np.savetxt(f"{outdir}/chain.txt", self.chain[:last + 1, :])
                if nc > 1:
                    np.save(f"{outdir}/chains.npy", self.chains[:, :last + 1])
                self._save_state(outdir, last + 1, eng)
        if flush_final:
            np.savetxt(f"{outdir}/chain.txt", self.chain[:self.iter + 1, :])
            if nc > 1:
                np.save(f"{outdir}/chains.npy", self.chains[:, :self.iter + 1])
            self._save_state(outdir, self.iter + 1, eng)
        b = eng.b.cpu().numpy()
        self._b = [b[p * eng.C, :eng.model.m[p]] for p in range(eng.P)]
        if eng.hyper is not None:
            self.aclength_hyper = eng.hyper_acl
            self.hyper_acceptance = eng.hyper.acceptance()
        return self.chain
