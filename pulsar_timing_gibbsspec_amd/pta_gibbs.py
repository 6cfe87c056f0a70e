"""``PTABlockGibbs`` — drop-in for the reference's multi-pulsar sampler.

Mirrors ``/root/reference/pta_gibbs.py:14-713`` for the common free-spectrum
(CURN) model with optional per-pulsar red free spectra drawn conditionally
(``redsample='conditional'``): same constructor, parameter plumbing, prior
parsing, per-pulsar gwid discovery, ``update_b`` / ``update_rho_params`` /
``update_hyper_params`` / ``sample`` surface and ``chain.txt`` output.  All
arithmetic runs on the GPU (engine.PTAChains); chains are batched
(``nchains``), chain 0 is written in the reference layout.

Outside the device hot path (raise NotImplementedError): Metropolis blocks —
white noise, ECORR, ``redsample='mh'`` hyper-parameters, ``hypersample='mh'``.
"""
from __future__ import annotations

import os
import sys
import time

import numpy as np
import torch

from . import _lib
from .engine import DeviceModel, PTAChains
from .pulsar_gibbs import _parse_uniform_bounds


class PTABlockGibbs(object):
    """Gibbs-based pulsar-timing periodogram analysis of a PTA on MI355X
    (van Haasteren & Vallisneri 2014)."""

    def __init__(self, pta, hypersample="conditional", redsample="mh", *, nchains=1, device=0,
                 seed=None):
        self.pta = pta
        self.hypersample = hypersample
        self.redsample = redsample
        self.nchains = int(nchains)
        if not np.any(["basis_ecorr" in key for key in self.pta._signal_dict.keys()]):
            print("ERROR: Gibbs outlier analysis must use basis_ecorr, not kernel ecorr")

        self._residuals = self.pta.get_residuals()
        xs = [p.sample() for p in pta.params]
        self._b = [np.zeros(self.pta.get_basis(xs)[ii].shape[1]) for ii in range(len(self.pta.pulsars))]
        self.TNT = []
        self.d = []

        ind = None
        for ct, par in enumerate([p.name for p in self.params]):
            if "rho" in par and "gw" in par:
                ind = ct
        if ind is None:
            raise UnboundLocalError("no common 'gw' ... 'rho' parameter in the PTA")
        lo, hi = _parse_uniform_bounds(self.params[ind].params[0])
        self.rhomin_gw, self.rhomax_gw = 10 ** (2 * lo), 10 ** (2 * hi)
        for ct, par in enumerate([p.name for p in self.params]):
            if "rho" in par and "red" in par:
                ind = ct
        lo, hi = _parse_uniform_bounds(self.params[ind].params[0])
        self.rhomin_red, self.rhomax_red = 10 ** (2 * lo), 10 ** (2 * hi)

        # per-pulsar GW basis indices (pta_gibbs.py:96-109)
        self.gwid = []
        for pname in self.pta.pulsars:
            ct = 0
            psigs = [sig for sig in self.pta.signals.keys() if pname in sig]
            for sig in psigs:
                Fmat = self.pta.signals[sig].get_basis()
                if "gw" in self.pta.signals[sig].name:
                    self.gwid.append(ct + np.arange(0, Fmat.shape[1]))
                if Fmat is not None and "red" not in sig:
                    ct += Fmat.shape[1]

        self.red_sig = []
        self.gw_sig = None
        for sig in self.pta.signals:
            if "red" in self.pta.signals[sig].name:
                self.red_sig.append(self.pta.signals[sig])
            if "gw" in self.pta.signals[sig].name:
                self.gw_sig = self.pta.signals[sig]

        self.ctx = _lib.Context(device, seed=np.random.SeedSequence(seed).generate_state(1, np.uint64)[0]
                                if seed is not None else 0)
        self._device_model = None
        self._engine = None

    # ------------------------------------------------------------ plumbing
    @property
    def params(self):
        return [p for p in self.pta.params]

    @property
    def param_names(self):
        ret = []
        for p in self.params:
            if p.size:
                for ii in range(0, p.size):
                    ret.append(p.name + "_{}".format(ii))
            else:
                ret.append(p.name)
        return ret

    def map_params(self, xs):
        ret = {}
        ct = 0
        for p in self.params:
            n = p.size if p.size else 1
            ret[p.name] = xs[ct: ct + n] if n > 1 else float(xs[ct])
            ct += n
        return ret

    def _indices(self, pred):
        return np.array([ct for ct, par in enumerate(self.param_names) if pred(par)])

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
        if hind.size and self.redsample != "conditional":
            raise NotImplementedError("redsample='mh' is outside the device hot path; use 'conditional'")
        if hind.size and hind.size != len(self.pta.pulsars) * (len(self.gwid[0]) // 2):
            raise NotImplementedError("per-pulsar red noise must be a free spectrum on the gw basis")
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

    def _new_engine(self, xs):
        self._check_supported()
        model = self._model(xs)
        hind = self.get_hyper_param_indices()
        red_col = hind.reshape(len(self.pta.pulsars), -1) if hind.size else None
        return PTAChains(model, len(self.param_names), self.get_rho_param_indices(), red_col,
                         (self.rhomin_gw, self.rhomax_gw), (self.rhomin_red, self.rhomax_red),
                         self.nchains, np.asarray(xs, float))

    # ------------------------------------------------------------ conditionals (single-call API)
    def _engine_at(self, xs):
        eng = self._engine or self._new_engine(xs)
        self._engine = eng
        eng.x.copy_(torch.as_tensor(np.asarray(xs, float), device=self.ctx.device).expand_as(eng.x))
        b = np.zeros((len(self._b), eng.model.ldb))
        for p, bb in enumerate(self._b):
            b[p, :bb.size] = bb
        eng.b.copy_(torch.as_tensor(np.repeat(b, eng.C, axis=0), device=self.ctx.device))
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
        if eng.red:
            _lib.check(lib.gs_phi_from_x(h, eng.C, eng.P * eng.n_f, _lib.ptr(eng.x), eng.n_param,
                                         _lib.ptr(eng.red_col), _lib.ptr(eng.irn)), "gs_phi_from_x")
        _lib.check(lib.gs_rho_curn(h, eng.P, eng.C, eng.n_f, _lib.ptr(eng.tau), _lib.ptr(eng.irn),
                                   eng.ngrid, _lib.ptr(eng.grid_gw), None, eng.it, 0, _lib.ptr(eng.x),
                                   eng.n_param, _lib.ptr(eng.gw_col), None), "gs_rho_curn")
        eng.it += 1
        return eng.x[0].cpu().numpy()

    def update_hyper_params(self, xs, iters=None):
        """Per-pulsar red free spectra | b, phi_gw (pta_gibbs.py:246-276), on the GPU."""
        if self.redsample != "conditional":
            raise NotImplementedError("redsample='mh' is outside the device hot path")
        eng = self._engine_at(xs)
        if not eng.red:
            return np.asarray(xs, float).copy()
        lib, h, m = self.ctx.lib, self.ctx.handle, eng.model
        _lib.check(lib.gs_tau(h, eng.P, eng.C, m.NF, m.ldb, _lib.ptr(m.fidx), _lib.ptr(eng.b), 0,
                              _lib.ptr(eng.tau)), "gs_tau")
        _lib.check(lib.gs_phi_from_x(h, eng.C, eng.n_f, _lib.ptr(eng.x), eng.n_param, _lib.ptr(eng.gw_col),
                                     _lib.ptr(eng.gwphi)), "gs_phi_from_x")
        _lib.check(lib.gs_rho_red(h, eng.P, eng.C, eng.n_f, _lib.ptr(eng.tau), _lib.ptr(eng.gwphi), eng.ngrid,
                                  _lib.ptr(eng.grid_red), None, eng.it, 0, _lib.ptr(eng.x), eng.n_param,
                                  _lib.ptr(eng.red_col), None), "gs_rho_red")
        eng.it += 1
        return eng.x[0].cpu().numpy()

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
        if resume and os.path.exists(f"{outdir}/chain.txt"):
            print("Resuming from previous run...")
            prev = np.atleast_2d(np.loadtxt(f"{outdir}/chain.txt"))
            start = prev.shape[0]
            self.chain[:start] = prev
            x0 = prev[-1]
        eng = self._new_engine(x0)
        self._engine = eng
        dev = self.ctx.device
        buf = torch.empty(save_every + 1, nc, npar, dtype=torch.float64, device=dev)
        tstart = time.time()
        ii = start
        if start > 0:                      # resume: redo sweep start-1 from its recorded state
            eng.it = start - 1
            eng.sweep()
            ii = start
        while ii < niter:
            nxt = min(niter, (ii // save_every + 1) * save_every + 1)
            for j in range(nxt - ii):
                eng.sweep(x_rec=buf[j])
            rows = buf[:nxt - ii].cpu().numpy()
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
        if flush_final:
            np.savetxt(f"{outdir}/chain.txt", self.chain[:self.iter + 1, :])
            if nc > 1:
                np.save(f"{outdir}/chains.npy", self.chains[:, :self.iter + 1])
        b = eng.b.cpu().numpy()
        self._b = [b[p * eng.C, :eng.model.m[p]] for p in range(eng.P)]
        if eng.info.cpu().numpy().any():
            print("WARNING: non-positive-definite Sigma encountered")
        return self.chain
