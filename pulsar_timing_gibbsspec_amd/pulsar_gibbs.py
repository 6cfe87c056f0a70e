"""``PulsarBlockGibbs`` — drop-in for the reference's single-pulsar sampler.

Mirrors ``/root/reference/pulsar_gibbs.py:14-710``: same constructor, same
parameter plumbing (``params``, ``param_names``, ``map_params``,
``get_*_indices``), same prior-bound parsing, same basis-index (gwid)
discovery, same ``update_b`` / ``update_gwrho_params`` / ``sample`` surface and
the same chain files.  The arithmetic runs on the GPU through the C-ABI:

* ``update_b``           -> gs_bdraw  (Cholesky draw; reference SVD draw :489-520)
* ``update_gwrho_params`` -> gs_rho_analytic (:206-216) — analytic branch
* ``sample``             -> gs_sweep_freespec, the whole loop body (:656-698) on device

* ``update_white_params`` -> gs_white_resid + gs_white_mh (:332-406), and with
  white noise sampled ``sample`` runs the per-sweep sequence of
  white.WhiteFreeSpectrumChains (per-chain TNT via gs_white_tnt, gs_prefix_sys,
  gs_bdraw_sys)

Extensions (keyword-only, reference-equivalent defaults): ``nchains``
(independent chains, chain 0 is written in the reference layout), ``device``,
``seed`` (Philox key).

* power-law intrinsic red noise: ``update_red_params`` /
  ``get_lnlikelihood_red`` -> gs_red_mh (:271-329, :549-566), rho|b -> gs_rho_gumbel
  (:218-236), and ``sample`` runs rednoise.RedNoiseChains.
* basis ECORR: ``update_ecorr_params`` (:409-486) with
  ``get_lnlikelihood`` = the marginalised likelihood (the notebook's definition; the .py
  calls it without defining it), ``update_b`` / ``get_lnlikelihood_fullmarg`` through the
  ECORR-eliminated Schur systems (ecorr.EcorrModel), and ``sample`` runs the notebook
  sampler's order (ECORR block, rho|b, gated b; ecorr.EcorrFreeSpectrumChains) where the
  .py prints 'ERROR: No ECORR for now...' and skips the block (:675-683).
"""
from __future__ import annotations

import os

import numpy as np
import torch

from . import _lib
from .diagnostics import white_aclength
from .ecorr import EcorrFreeSpectrumChains, EcorrModel, EcorrWhiteChains
from .engine import DeviceModel, FreeSpectrumChains, HistoryStreamer, check_handoff, grid3
from .plumbing import (basis_layout, expand_names, last_match, matching_indices, power_bounds,
                       uniform_bounds, vector_to_dict)
from .rednoise import (DE_BUFFER, RED_STEPS, RedJumps, RedNoiseChains, powerlaw_loglinear,
                       warmup as red_warmup)
from .white import MAX_W, WhiteFreeSpectrumChains, WhiteNoiseModel, white_kind


# Global chain id base of the single-call API (update_b, update_white_params, ...): its
# Philox counters (slot, sweep, chain, pulsar/event) then never coincide with those of a
# sample() run, whose chains are 0 .. nchains - 1 (the warm-up's draws were
# being reused by chain 0's first sweeps).
HOST_CHAIN = 1 << 31


def resolve_seed(seed):
    """(seed, Philox key) of a sampler.  seed=None draws fresh OS entropy, as the reference's
    unseeded global np.random does, so independent jobs never repeat each other's chains; the
    drawn seed is kept on the sampler (``.seed``) so a run can be reproduced."""
    if seed is None:
        seed = int(np.random.SeedSequence().entropy % (1 << 63))
    return int(seed), int(np.random.SeedSequence(int(seed)).generate_state(1, np.uint64)[0])


def save_rows(s, outdir, n, chains=False, bchains=False):
    """Write rows [:n] of s.chain / s.bchain to chain.npy / bchain.npy (the reference's periodic
    save, pulsar_gibbs.py:701-710) and, for multi-chain runs, the leading-chain-axis chains.npy /
    bchains.npy beside them."""
    np.save(f"{outdir}/chain.npy", s.chain[:n, :])
    np.save(f"{outdir}/bchain.npy", s.bchain[:n, :])
    if chains:
        np.save(f"{outdir}/chains.npy", s.chains[:, :n])
    if bchains:
        np.save(f"{outdir}/bchains.npy", s.bchains[:, :n])


def sample_free_spectrum(samplers, model, xs_list, outdirs, niter, resume, save_every, psr_base=0,
                         record_bchains=None):
    """The free-spectrum sample loop (PulsarBlockGibbs.sample, pulsar_gibbs.py:620-710) for
    one or many pulsars at once: pulsar p of ``model`` is ``samplers[p]``'s PTA, its chains
    are systems p*nchains .. p*nchains + nchains - 1 of one FreeSpectrumChains run (the
    fused sweep kernel), and its files go to ``outdirs[p]``.

    Per pulsar, exactly the reference's layout: chain row ii = state BEFORE sweep ii (row 0
    = xs, bchain[0] = 0); chain.npy / bchain.npy rewritten with rows [:ii+1] at ii % 100 == 0,
    ii > 0 (pulsar_gibbs.py:701-710); with nchains > 1 also chains.npy / bchains.npy.
    Resume continues from the shortest saved chain of the pulsars: the recorded (x, b) of
    row start-1 are restored and sweep start-1 re-run with its own Philox counters, so a
    resumed run reproduces the uninterrupted one bit for bit.

    record_bchains: keep every chain's b history on the host (``bchains``, bchains.npy);
    default only for nchains <= 16 -- 4096 chains x 10^4 sweeps of b are 25 GB, and chain 0's
    b (the reference's bchain) is what the reference layout needs.  Without it only chain 0's
    b rows cross PCIe (the rest are recorded in HBM only)."""
    P = len(samplers)
    nc = samplers[0].nchains
    ctx = model.ctx
    dev = ctx.device
    rhomin, rhomax = samplers[0].rhomin, samplers[0].rhomax
    m = [int(v) for v in model.m]
    n_f = model.NF // 2
    if record_bchains is None:
        record_bchains = nc <= 16
    allb = nc > 1 and bool(record_bchains)
    for s in samplers:
        s.chain = np.zeros((niter, n_f))
        s.bchain = np.zeros((niter, len(s._b)))
        s.chains = np.zeros((nc, niter, n_f)) if nc > 1 else None
        s.bchains = np.zeros((nc, niter, len(s._b))) if allb else None
        s.iter = 0
    start = 0
    multi_x = multi_b = False
    if resume and all(os.path.exists(f"{o}/chain.npy") for o in outdirs):
        print("Resuming from previous run...")
        prev = [(np.load(f"{o}/chain.npy"), np.load(f"{o}/bchain.npy")) for o in outdirs]
        start = min(min(c.shape[0], b.shape[0]) for c, b in prev)
        for s, (c0, b0) in zip(samplers, prev):
            s.chain[:start] = c0[:start]
            s.bchain[:start] = b0[:start]
        # every chain's x rows from chains.npy whenever it is there (nc > 1), whether or not
        # every chain's b was kept; b rows from bchains.npy when it was (record_bchains)
        if nc > 1 and all(os.path.exists(f"{o}/chains.npy") for o in outdirs):
            prevc = [np.load(f"{o}/chains.npy") for o in outdirs]
            multi_x = all(c.shape[0] == nc and c.shape[1] >= start for c in prevc)
            if multi_x:
                for s, c0 in zip(samplers, prevc):
                    s.chains[:, :start] = c0[:, :start]
        if multi_x and allb and all(os.path.exists(f"{o}/bchains.npy") for o in outdirs):
            prevb = [np.load(f"{o}/bchains.npy") for o in outdirs]
            multi_b = all(b.shape[0] == nc and b.shape[1] >= start for b in prevb)
            if multi_b:
                for s, b0 in zip(samplers, prevb):
                    s.bchains[:, :start] = b0[:, :start]
    x0 = np.concatenate([np.broadcast_to(np.asarray(x, float), (nc, n_f)) for x in xs_list])
    ctx.set_option(_lib.OPT_PSR_BASE, int(psr_base))
    runner = FreeSpectrumChains(model, rhomin, rhomax, nc, x0)
    if start > 0:
        for p, s in enumerate(samplers):
            rows = slice(p * nc, (p + 1) * nc)
            runner.x[rows] = torch.as_tensor(s.chains[:, start - 1] if multi_x else s.chain[start - 1], device=dev)
            runner.b[rows, :m[p]] = torch.as_tensor(s.bchains[:, start - 1] if multi_b else s.bchain[start - 1],
                                                    device=dev)
        if multi_x and not multi_b:
            # every chain's x is restored but only chain 0's b was kept (bchain.npy, the
            # reference's file): chains 1.. get b drawn from b | x at their own x (Philox event
            # GS_EV_B0 of sweep start-1), a valid Gibbs state; chain 0 keeps its recorded b, so
            # its continuation is the uninterrupted run's bit for bit
            ph = torch.pow(10.0, -2.0 * runner.x).repeat_interleave(2, dim=1).contiguous()
            bnew, _ = model.bdraw(ph, nc, sweep=start - 1, event=_lib.EV_B0, chain_base=runner.chain_base)
            keep = torch.zeros(model.P, nc, 1, dtype=torch.bool, device=dev)
            keep[:, 0] = True
            runner.b.copy_(torch.where(keep, runner.b.view(model.P, nc, -1),
                                       bnew.view(model.P, nc, -1)).view_as(runner.b))
        runner.it = start - 1
        runner.run(1, record=False)        # re-run sweep start-1: row start-1's successor
    runner.it = max(runner.it, start)
    blk = max(1, save_every) + 1
    # block k+1's sweeps run while block k's rows reach pinned host memory: the kernel writes
    # every chain's x rows and chain 0's b rows (GS_OPT_BREC_CHAINS = 1; the reference's bchain)
    # straight into the pinned slots; every chain's b (record_bchains) goes through HBM and the
    # copy engine
    bk = nc if (allb or nc == 1) else 1
    streamer = HistoryStreamer(ctx, [(blk, P * nc, n_f), (blk, P * bk, model.ldb)], direct=[True, not allb])
    bstride = bk
    # failed (non-PD) draws, surfaced per block as they happen: the kernels keep b and count
    # (gs_ctx_set_fail_counts); each block's counts reach pinned memory behind the block
    fc_host = [torch.zeros(P * nc, dtype=torch.int32, pin_memory=True) for _ in range(2)]
    info_host = [torch.zeros(P * nc, dtype=torch.int32, pin_memory=True) for _ in range(2)]
    fc_ev = [torch.cuda.Event(), torch.cuda.Event()]
    fc_seen = [int(runner.fail_count.sum())]

    def consume(slot, ii, nxt):
        xh, bh = (t.numpy() for t in streamer.fetch(slot))
        fc_ev[slot].synchronize()
        # a chain whose hand-off wait expired (info = -1) was not advanced: fail loudly
        check_handoff(info_host[slot])
        tot = int(fc_host[slot].sum())
        if tot > fc_seen[0]:
            bad = np.nonzero(fc_host[slot].numpy())[0]
            print(f"WARNING: sweeps {ii}..{nxt - 1}: {tot - fc_seen[0]} b draws hit a non-positive-definite "
                  f"Sigma; those chains KEEP their previous b -- unlike the reference, whose LinAlgError "
                  f"branch (pulsar_gibbs.py:507-516) redraws b from a QR/SVD of Sigma with the wrong "
                  f"covariance (SURVEY Appendix A.7); systems so far: {bad[:8].tolist()}"
                  f"{' ...' if bad.size > 8 else ''}")
            fc_seen[0] = tot
        last = nxt - 1
        save = last % save_every == 0 and last > 0
        for p, (s, o) in enumerate(zip(samplers, outdirs)):
            xp = xh[:, p * nc:(p + 1) * nc]
            bp = bh[:, p * bstride:(p + 1) * bstride, :m[p]]
            s.chain[ii:nxt] = xp[:, 0]
            s.bchain[ii:nxt] = bp[:, 0]
            if nc > 1:
                s.chains[:, ii:nxt] = np.moveaxis(xp, 1, 0)
            if allb:
                s.bchains[:, ii:nxt] = np.moveaxis(bp, 1, 0)
            s.iter = last
            if save:
                save_rows(s, o, last + 1, nc > 1, allb)

    ii, slot, pending = start, 0, None
    while ii < niter:
        nxt = min(niter, (ii // save_every + 1) * save_every + 1)
        n = nxt - ii
        xr, br = streamer.buffers(slot, n)
        runner.run(n, x_rec=xr, b_rec=br, record_b_chains=bk)
        with torch.cuda.stream(ctx.stream):
            fc_host[slot].copy_(runner.fail_count, non_blocking=True)
            info_host[slot].copy_(runner.info, non_blocking=True)
            fc_ev[slot].record(ctx.stream)
        streamer.submit(slot, n)
        if pending is not None:
            consume(*pending)
        pending = (slot, ii, nxt)
        slot ^= 1
        ii = nxt
    if pending is not None:
        consume(*pending)
    b_end = runner.b.cpu().numpy()
    for p, s in enumerate(samplers):
        s._b = b_end[p * nc, :m[p]].copy()
        s._runner = runner
    return runner


class PulsarBlockGibbs(object):
    """Gibbs-based pulsar-timing periodogram analysis on MI355X.

    van Haasteren & Vallisneri (2014), PRD 90, 104012 (arXiv:1407.1838);
    blocked Gibbs: b | rho, data and rho | b.
    """

    def __init__(self, pta, hypersample="conditional", ecorrsample="mh", psr=None, *,
                 nchains=1, device=0, seed=None, ctx=None):
        self.pta = pta
        self.pulsar_name = pta.pulsars[0]
        self.hypersample = hypersample
        self.ecorrsample = ecorrsample
        self.nchains = int(nchains)

        # kernel ECORR is not a Gibbs block (pulsar_gibbs.py:65-68)
        if any("EcorrKernelNoise" in type(pta.signals[k]).__name__ for k in pta.signals):
            raise TypeError("Gibbs outlier analysis must use basis_ecorr, not kernel ecorr")

        self._residuals = pta.get_residuals()[0]
        self._b = np.zeros(pta.get_basis([p.sample() for p in pta.params])[0].shape[1])
        self.TNT = None
        self.d = None

        # free-spectrum prior: the last 'gw' + 'rho' parameter (pulsar_gibbs.py:82-87)
        ind = last_match([p.name for p in self.params], lambda n: "rho" in n and "gw" in n)
        if ind is None:
            raise UnboundLocalError("no gw free-spectrum ('gw' ... 'rho') parameter in the PTA")
        self.rhomin, self.rhomax = power_bounds(self.params[ind].params[0])

        # columns of the gw (and ECORR) blocks in T (pulsar_gibbs.py:89-109)
        self.gwid, self.ecid, self.b_param_names, ncol = basis_layout(pta.signals)
        print("Basis count is good" if ncol == pta.get_basis()[0].shape[1] else
              "WARNING: Miscounted basis entries. Maybe red noise and GW do not share a design matrix.")

        if self.ecid is not None:
            # ECORR prior: the last 'ecorr' parameter (pulsar_gibbs.py:111-118)
            ind = last_match([p.name for p in self.params], lambda n: "ecorr" in n)
            self.ecorrmin, self.ecorrmax = power_bounds(self.params[ind].params[0])
            if self.ecorrsample == "conditional":
                # the reference's epoch selection needs enterprise's selections.by_backend
                # (:121-127) and its conditional draw is commented out ('NEEDS TO BE FIXED')
                raise NotImplementedError("ecorrsample='conditional' is not implemented in the reference")

        # the last signal named 'red' / 'gw' (pulsar_gibbs.py:130-136)
        sigs = [pta.signals[k] for k in pta.signals]
        self.red_sig = next((s for s in reversed(sigs) if "red" in s.name), None)
        self.gw_sig = next((s for s in reversed(sigs) if "gw" in s.name), None)

        # ---- device side (the context is created on first use: the plumbing above
        # needs no GPU)
        self.seed, self._key = resolve_seed(seed)
        self._device = device
        self._ctx = ctx
        self._ndraw = 0
        self._device_model = None

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

    def get_gwrho_param_indices(self):
        return self._indices(lambda par: "rho" in par)

    def get_red_param_indices(self):
        return self._indices(lambda par: "log10_A" in par or "gamma" in par)

    def get_efacequad_indices(self):
        return self._indices(lambda par: "efac" in par or "equad" in par)

    def get_ecorr_indices(self):
        return self._indices(lambda par: "ecorr" in par)

    def get_lnprior(self, params):
        params = params if isinstance(params, dict) else self.map_params(params)
        return np.sum([p.get_logpdf(params=params) for p in self.params])

    # ------------------------------------------------------------ device model
    def _model(self, xs):
        """TNT/d + fixed-prior prefix on device; rebuilt when N changes."""
        params = self.map_params(xs)
        Nvec = self.pta.get_ndiag(params)[0]
        if self._device_model is not None and np.array_equal(Nvec, self._model_N):
            return self._device_model
        T = self.pta.get_basis(params)[0]
        phiinv = self.pta.get_phiinv(params, logdet=False)[0]
        mask = np.ones(T.shape[1], bool)
        mask[self.gwid] = False
        self._device_model = DeviceModel(self.ctx, [T], [Nvec], [self._residuals], [self.gwid],
                                         [phiinv[mask]])
        self._model_N = Nvec.copy()
        self._phfix = phiinv[mask].copy()
        return self._device_model

    def _phiinv_F(self, xs):
        params = self.map_params(xs)
        phiinv = self.pta.get_phiinv(params, logdet=False)[0]
        mask = np.ones(phiinv.size, bool)
        mask[self.gwid] = False
        if self._device_model is not None and not np.array_equal(phiinv[mask], self._phfix):
            raise NotImplementedError("phiinv of the non-free-spectrum columns changed between draws; "
                                      "only fixed-prior columns are supported outside gwid")
        return phiinv[self.gwid]

    def get_lnlikelihood_fullmarg(self, xs):
        """Marginalised likelihood (pulsar_gibbs.py:569-610) on the device: the prefix
        model block + one augmented tile factorisation (gs_lnlike_marg); -inf when
        Sigma is not positive definite (the reference's LinAlgError branch, :598-599).
        With basis ECORR: the ECORR-eliminated Schur system (ecorr.EcorrModel.lnlike)."""
        if self.ecid is not None:
            em = self._ecorr_model1(xs)
            x = torch.as_tensor(np.asarray(xs, float)[None, :], device=self.ctx.device).contiguous()
            ph = torch.as_tensor(np.ascontiguousarray(self._ecorr_phiinv_F(xs))[None], device=self.ctx.device)
            const = self._ecorr_lnl_const(xs) if self._ecorr_white() else None
            return float(em.lnlike(x, ph, lnl_const=const)[0])
        model = self._model(xs)
        ph = torch.as_tensor(np.ascontiguousarray(self._phiinv_F(xs))[None], device=self.ctx.device)
        lnl, info = model.lnlike_marg(ph, 1)
        return -np.inf if int(info[0]) else float(lnl[0])

    def get_lnlikelihood(self, xs):
        """The likelihood update_ecorr_params calls (pulsar_gibbs.py:420, 463) and the .py
        never defines; the notebook's get_lnlikelihood is get_lnlikelihood_fullmarg's code."""
        return self.get_lnlikelihood_fullmarg(xs)

    # ------------------------------------------------------------ basis ECORR (8f-4)
    def _ecorr_loop(self):
        extra = [n for n in self.param_names if "rho" not in n]
        return (self.ecid is not None and any("ecorr" in n for n in extra)
                and all(("ecorr" in n or "efac" in n or "equad" in n) for n in extra))

    def _ecorr_white(self):
        return self.ecid is not None and self.get_efacequad_indices().size > 0

    def _ecorr_structure(self, xs):
        """(eind, epoch_backend, emin, emax) through the PTA contract: the ECORR columns
        whose phi moves with each ECORR parameter; phi_E = 10**(2 log10_ecorr) is verified."""
        eind = self.get_ecorr_indices()
        x0 = np.asarray(xs, float)
        ec = np.asarray(self.ecid)
        ph0 = 1.0 / self.pta.get_phiinv(self.map_params(x0), logdet=False)[0][ec]
        ebk = np.full(ec.size, -1, np.int64)
        for k, j in enumerate(eind):
            xp = x0.copy()
            xp[j] += 0.5
            mv = 1.0 / self.pta.get_phiinv(self.map_params(xp), logdet=False)[0][ec] != ph0
            if (ebk[mv] != -1).any():
                raise NotImplementedError("ECORR selections overlap")
            ebk[mv] = k
        if (ebk == -1).any():
            raise NotImplementedError("ECORR epoch column not driven by any ECORR parameter")
        want = np.array([10.0 ** (2.0 * float(x0[j])) for j in eind])[ebk]
        if np.max(np.abs(ph0 - want) / want) > 1e-12:
            raise NotImplementedError("ECORR phi is not 10**(2 log10_ecorr) per epoch")
        bounds = []
        for p in self.params:
            lo, hi = uniform_bounds(p)
            bounds += [(lo, hi)] * (p.size or 1)
        emin = np.array([bounds[j][0] for j in eind])
        emax = np.array([bounds[j][1] for j in eind])
        return eind, ebk, emin, emax

    def _ecorr_model(self, xs, n_chain, per_chain=False):
        params = self.map_params(xs)
        T = self.pta.get_basis(params)[0]
        Nvec = self.pta.get_ndiag(params)[0]
        phiinv = self.pta.get_phiinv(params, logdet=False)[0]
        eind, ebk, emin, emax = self._ecorr_structure(xs)
        fixed = np.setdiff1d(np.arange(T.shape[1]), np.concatenate([self.ecid, self.gwid]))
        return EcorrModel(self.ctx, T, Nvec, self._residuals, self.ecid, ebk, self.gwid, eind, emin, emax,
                          len(xs), n_chain, phiinv_fixed=phiinv[fixed], per_chain=per_chain)

    def _ecorr_model1(self, xs):
        """The 1-chain ECORR model; with white noise sampled its operands are rebuilt from
        the TNT of xs's N on every call (the reference's TNT reset + recompute)."""
        if getattr(self, "_em1", None) is None:
            self._em1 = self._ecorr_model(xs, 1, per_chain=self._ecorr_white())
            if self._ecorr_white():
                self._wm1e = self._white_model(xs, 1)
        if self._ecorr_white():
            x = torch.as_tensor(np.asarray(xs, float)[None, :], device=self.ctx.device).contiguous()
            self._wm1e.tnt(x, x.shape[1])
            self._em1.gather(self._wm1e.TNT, self._wm1e.d, self._wm1e.tnt_cstride, self._wm1e.d_cstride)
        return self._em1

    def _ecorr_lnl_const(self, xs):
        """-1/2 (sum log N + r^T N^-1 r) + 1/2 sum_M log phiinv_M at xs's white noise."""
        params = self.map_params(xs)
        N = self.pta.get_ndiag(params)[0]
        phiinv = self.pta.get_phiinv(params, logdet=False)[0]
        fixed = np.setdiff1d(np.arange(phiinv.size), np.concatenate([self.ecid, self.gwid]))
        r = self._residuals
        return float(-0.5 * (np.sum(np.log(N)) + np.sum(r ** 2 / N)) + 0.5 * np.sum(np.log(phiinv[fixed])))

    def _ecorr_phiinv_F(self, xs):
        return self.pta.get_phiinv(self.map_params(xs), logdet=False)[0][self.gwid]

    def update_ecorr_params(self, xs, iters=None, inj=None):
        """Basis-ECORR Metropolis block (pulsar_gibbs.py:409-486) on the GPU: with ``iters``
        the warm-up (cov_ecorr, sigma_ecorr, svd_ecorr and aclength_ecorr from acor of the
        proposal chain after 100 steps, :448-451), else ``aclength_ecorr`` steps.  ``inj``
        (steps, 4): injected (scale, parameter index within eind, normal, uniform)."""
        dev = self.ctx.device
        em = self._ecorr_model1(xs)
        x = torch.as_tensor(np.asarray(xs, float)[None, :], device=dev).contiguous()
        ph = torch.as_tensor(np.ascontiguousarray(self._ecorr_phiinv_F(xs))[None], device=dev)
        n = int(iters) if iters is not None else int(self.aclength_ecorr)
        q_rec = torch.empty(n, 1, em.n_bk, dtype=torch.float64, device=dev) if iters is not None else None
        it = None if inj is None else torch.as_tensor(np.asarray(inj, float).reshape(n, 1, 4), device=dev)
        em.mh(x, ph, n, sweep=self._ndraw, chain_base=HOST_CHAIN, inj=it, q_rec=q_rec)
        self._ndraw += 1
        if iters is not None:
            short_chain = q_rec[:, 0].cpu().numpy()
            self.cov_ecorr = np.cov(short_chain[100:, :], rowvar=False)
            self.sigma_ecorr = np.diag(np.atleast_2d(self.cov_ecorr)) ** 0.5
            self.svd_ecorr = np.linalg.svd(np.atleast_2d(self.cov_ecorr))
            self.aclength_ecorr = white_aclength(short_chain)
        return x[0].cpu().numpy()

    # ------------------------------------------------------------ white noise
    def _white_structure(self, xs):
        """Per-TOA sigma^2, backend groups and the white parameter table, discovered
        through the PTA contract alone (get_ndiag): sigma^2 = N at efac = 1 and
        negligible equads; the TOAs a parameter acts on = where N moves when it moves.
        Verified against get_ndiag at xs before use."""
        wind = self.get_efacequad_indices()
        names = self.param_names
        x0 = np.asarray(xs, float).copy()
        base = x0.copy()
        kinds = [white_kind(names[j]) for j in wind]
        for j, k in zip(wind, kinds):
            base[j] = 1.0 if k == 0 else -40.0
        N0 = self.pta.get_ndiag(self.map_params(base))[0]
        masks = []
        for j, k in zip(wind, kinds):
            xp = base.copy()
            xp[j] = 2.0 if k == 0 else -5.0
            masks.append(self.pta.get_ndiag(self.map_params(xp))[0] != N0)
        groups = []
        bk = np.full(N0.size, -1, np.int64)
        wl = []
        bounds = {}
        for p in self.params:
            lo, hi = uniform_bounds(p)
            for n in ([p.name] if not p.size else [f"{p.name}_{i}" for i in range(p.size)]):
                bounds[n] = (lo, hi)
        for j, k, mk in zip(wind, kinds, masks):
            key = mk.tobytes()
            if key not in groups:
                if (bk[mk] != -1).any():
                    raise NotImplementedError("white-noise selections overlap")
                groups.append(key)
                bk[mk] = len(groups) - 1
            wl.append((int(j), k, groups.index(key), *bounds[names[j]]))
        if (bk == -1).any():
            bk[bk == -1] = len(groups)
        if len(wl) > MAX_W:
            raise NotImplementedError(f"more than {MAX_W} white parameters")
        # verify the device formula N = efac^2 (sigma^2 + t2equad^2) + tnequad^2 at xs
        nb = int(bk.max()) + 1
        ef, t2, tn = np.ones(nb), np.zeros(nb), np.zeros(nb)
        for (j, k, g, _, _) in wl:
            if k == 0:
                ef[g] = x0[j] ** 2
            elif k == 1:
                tn[g] = 10.0 ** (2.0 * x0[j])
            else:
                t2[g] = 10.0 ** (2.0 * x0[j])
        N = ef[bk] * (N0 + t2[bk]) + tn[bk]
        Nref = self.pta.get_ndiag(self.map_params(x0))[0]
        if np.max(np.abs(N - Nref) / Nref) > 1e-12:
            raise NotImplementedError("white-noise model is not efac/equad per backend")
        return N0, bk, wl

    def _white_model(self, xs, n_chain, cols=None):
        params = self.map_params(xs)
        sigma2, bk, wl = self._white_structure(xs)
        T = self.pta.get_basis(params)[0]
        if cols is not None:   # the R columns of a basis-ECORR model (TNT_RR only)
            pos = {c: i for i, c in enumerate(cols)}
            return WhiteNoiseModel(self.ctx, [np.ascontiguousarray(T[:, cols])], [self._residuals],
                                   [np.sqrt(sigma2)], [bk], [np.array([pos[c] for c in self.gwid])],
                                   [np.full(len(cols) - len(self.gwid), 1e-40)], [wl], n_chain, prefix=False)
        phiinv = self.pta.get_phiinv(params, logdet=False)[0]
        mask = np.ones(T.shape[1], bool)
        mask[self.gwid] = False
        self._phfix = phiinv[mask].copy()
        # with basis ECORR the per-chain Schur systems are factored by ecorr.EcorrModel: the
        # white model only supplies TNT_c / d_c, residuals and the white MH (prefix=False)
        return WhiteNoiseModel(self.ctx, [T], [self._residuals], [np.sqrt(sigma2)], [bk], [self.gwid],
                               [phiinv[mask]], [wl], n_chain, prefix=self.ecid is None)

    def update_white_params(self, xs, iters=None, inj=None):
        """White-noise Metropolis block (pulsar_gibbs.py:332-406) on the GPU: with
        ``iters`` the warm-up (sets aclength_white from acor of the proposal chain,
        cov_white, sigma_white, svd_white), else ``aclength_white`` steady-state steps.
        ``inj`` (steps, 4): injected (scale, parameter index within wind, normal, uniform)."""
        dev = self.ctx.device
        if getattr(self, "_wm1", None) is None:
            self._wm1 = self._white_model(xs, 1)
        wm = self._wm1
        wind = self.get_efacequad_indices()
        x = torch.as_tensor(np.asarray(xs, float)[None, :], device=dev).contiguous()
        b = torch.zeros(1, wm.ldb, dtype=torch.float64, device=dev)
        b[0, :self._b.size] = torch.as_tensor(self._b, device=dev)
        wm.resid(b)
        n = int(iters) if iters is not None else int(self.aclength_white)
        q_rec = torch.empty(n, 1, MAX_W, dtype=torch.float64, device=dev) if iters is not None else None
        it = None if inj is None else torch.as_tensor(np.asarray(inj, float).reshape(n, 1, 4), device=dev)
        wm.mh(x, x.shape[1], n, self._ndraw, chain_base=HOST_CHAIN, inj=it, q_rec=q_rec)
        self._ndraw += 1
        if iters is not None:
            short_chain = q_rec[:, 0, :wind.size].cpu().numpy()
            self.cov_white = np.cov(short_chain[100:, :], rowvar=False)
            self.sigma_white = np.diag(np.atleast_2d(self.cov_white)) ** 0.5
            self.svd_white = np.linalg.svd(np.atleast_2d(self.cov_white))
            self.aclength_white = white_aclength(short_chain)
        return x[0].cpu().numpy()

    # ------------------------------------------------------------ conditionals
    def update_b(self, xs, z=None):
        """b | rho, data (pulsar_gibbs.py:489-520) on the GPU.

        ``z`` (optional, length m): standard normals in the Cholesky draw's
        coordinates (parity mode); default: device Philox.  With basis ECORR: the
        ECORR-eliminated draw (ecorr.EcorrModel.bdraw; z by original column)."""
        if self.ecid is not None:
            dev = self.ctx.device
            em = self._ecorr_model1(xs)
            x = torch.as_tensor(np.asarray(xs, float)[None, :], device=dev).contiguous()
            ph = torch.as_tensor(np.ascontiguousarray(self._ecorr_phiinv_F(xs))[None], device=dev)
            zt = None if z is None else torch.as_tensor(np.asarray(z, float)[None, :em.m], device=dev).contiguous()
            b = torch.zeros(1, em.m, dtype=torch.float64, device=dev)
            em.bdraw(x, ph, b, z=zt, sweep=self._ndraw, first=False, chain_base=HOST_CHAIN)
            self._ndraw += 1
            if int(em.binfo[0]) != 0:
                raise np.linalg.LinAlgError(f"Sigma not positive definite (leading minor {int(em.binfo[0])})")
            return b[0].cpu().numpy()
        model = self._model(xs)
        self.TNT, self.d = model.tnt_host(0)
        dev = self.ctx.device
        ph = torch.as_tensor(self._phiinv_F(xs)[None, :], dtype=torch.float64, device=dev)
        zt = None if z is None else torch.as_tensor(np.asarray(z, float)[None, :model.ldb],
                                                    dtype=torch.float64, device=dev)
        b, info = model.bdraw(ph, 1, z=zt, sweep=self._ndraw, event=_lib.EV_USER, chain_base=HOST_CHAIN)
        self._ndraw += 1
        if int(info[0]) != 0:
            raise np.linalg.LinAlgError(f"Sigma not positive definite (leading minor {int(info[0])})")
        return b[0, :model.m[0]].cpu().numpy()

    def update_gwrho_params(self, xs, u=None):
        """rho | b (pulsar_gibbs.py:199-268) on the GPU: the analytic draw, or with an
        intrinsic red signal the grid + Gumbel-max draw (:218-234; ``u``: the (n_f, 1000)
        uniforms behind the Gumbels in parity mode)."""
        gwind = self.get_gwrho_param_indices()
        xnew = xs.copy()
        if self.hypersample != "conditional":
            print("ERROR: Only conditional draws on rho for now...")
            return xnew
        dev = self.ctx.device
        n_f = len(self.gwid) // 2
        b = torch.as_tensor(self._b[None, :], dtype=torch.float64, device=dev)
        fidx = torch.as_tensor(np.asarray(self.gwid, np.int32)[None, :], device=dev)
        if self.red_sig is not None:
            irn = np.array(self.red_sig.get_phi(self.map_params(xnew)))[::2]        # :223
            tau = torch.empty(n_f, 1, dtype=torch.float64, device=dev)
            _lib.check(self.ctx.lib.gs_tau(self.ctx.handle, 1, 1, 2 * n_f, b.shape[1], _lib.ptr(fidx),
                                           _lib.ptr(b), 1, _lib.ptr(tau)), "gs_tau")
            irt = torch.as_tensor(np.ascontiguousarray(irn[:, None]), dtype=torch.float64, device=dev)
            ut = None if u is None else torch.as_tensor(np.ascontiguousarray(np.asarray(u, float)[None]),
                                                        dtype=torch.float64, device=dev)
            x = torch.empty(1, n_f, dtype=torch.float64, device=dev)
            cols = torch.arange(n_f, dtype=torch.int32, device=dev)
            grid = grid3(self.rhomin, self.rhomax, device=dev)
            _lib.check(self.ctx.lib.gs_rho_gumbel(self.ctx.handle, 1, n_f, _lib.ptr(tau), _lib.ptr(irt), 1000,
                                                  _lib.ptr(grid), _lib.ptr(ut), self._ndraw, HOST_CHAIN, _lib.ptr(x),
                                                  n_f, _lib.ptr(cols), None), "gs_rho_gumbel")
            self._ndraw += 1
            xnew[gwind] = x[0].cpu().numpy()
            return xnew
        ut = None if u is None else torch.as_tensor(np.asarray(u, float)[None, :], dtype=torch.float64,
                                                    device=dev)
        x = torch.empty(1, n_f, dtype=torch.float64, device=dev)
        _lib.check(self.ctx.lib.gs_rho_analytic(self.ctx.handle, 1, 1, 2 * n_f, b.shape[1], _lib.ptr(fidx),
                                                _lib.ptr(b), _lib.ptr(ut), self._ndraw, HOST_CHAIN, self.rhomin,
                                                self.rhomax, _lib.ptr(x), n_f), "gs_rho_analytic")
        self._ndraw += 1
        xnew[gwind] = x[0].cpu().numpy()
        return xnew

    # ------------------------------------------------------------ power-law red noise (8f-2)
    def _red_setup(self, xs):
        """(ia, ig, lnphi, bounds): the log10_A / gamma indices, the power law's log-linear
        coefficients probed from red_sig.get_phi, and their Uniform prior bounds."""
        if getattr(self, "_red_info", None) is not None:
            return self._red_info
        rind = self.get_red_param_indices()
        names = self.param_names
        ia = [i for i in rind if "log10_A" in names[i]]
        ig = [i for i in rind if "gamma" in names[i]]
        if len(rind) != 2 or len(ia) != 1 or len(ig) != 1:
            raise NotImplementedError(f"power-law red noise needs one log10_A and one gamma, got "
                                      f"{[names[i] for i in rind]}")
        ia, ig = int(ia[0]), int(ig[0])
        x = np.asarray(xs, float).copy()

        def phi_of(la, ga):
            x[ia], x[ig] = la, ga
            return np.array(self.red_sig.get_phi(self.map_params(x)))[::2]
        lnphi = powerlaw_loglinear(phi_of)
        by_index = [p for p in self.params for _ in range(p.size or 1)]
        bounds = (uniform_bounds(by_index[ia]), uniform_bounds(by_index[ig]))
        self._red_info = (ia, ig, lnphi, bounds)
        return self._red_info

    def _param_bounds(self):
        lo, hi = [], []
        for p in self.params:
            a, b = uniform_bounds(p)
            lo += [a] * (p.size or 1)
            hi += [b] * (p.size or 1)
        return np.array(lo), np.array(hi)

    def _red_engine(self, xs, n_chain, jumps=None, x_first=None, chain_base=0):
        ia, ig, lnphi, bounds = self._red_setup(xs)
        if jumps is None:
            jumps = getattr(self, "_red_jumps", None) or RedJumps(np.eye(2) * 0.01, np.zeros((0, 2)), bounds,
                                                                  self.ctx.device)
        return RedNoiseChains(self._model(xs), len(xs), self.get_gwrho_param_indices(),
                              (ia, ig), lnphi, jumps, self.rhomin, self.rhomax, n_chain, xs, x_first=x_first,
                              chain_base=chain_base)

    def get_lnlikelihood_red(self, xs):
        """get_lnlikelihood_red (pulsar_gibbs.py:549-566) on the device at (xs, self._b)."""
        eng = self._red_engine(xs, 1)
        eng.b[0, :len(self._b)] = torch.as_tensor(self._b, device=self.ctx.device)
        return float(eng.lnlike_red()[0])

    def update_red_params(self, xs, iters=None):
        """update_red_params (pulsar_gibbs.py:271-329).  iters: the sweep-0 warm-up on the
        device's marginalised likelihood (rednoise.warmup), which learns the red block's
        proposal covariance and DE buffer and returns the joint step's state; None: one
        20-step Metropolis block on the red-only likelihood (gs_red_mh)."""
        rind = self.get_red_param_indices()
        xnew = np.asarray(xs, float).copy()
        ia, ig, _, bounds = self._red_setup(xnew)
        if iters is not None:
            lo, hi = self._param_bounds()
            rng = np.random.default_rng(np.random.SeedSequence([int(self.ctx.seed), 0x7ed]))

            def lnprob(x):
                return self.get_lnlikelihood_fullmarg(x) + self.get_lnprior(x)
            x1, cov, chain = red_warmup(lnprob, xnew, int(iters), rng, lo, hi)
            sub = [ia, ig]
            self.cov_red = cov[np.ix_(sub, sub)]
            de = chain[-DE_BUFFER:][:, sub] if len(chain) else np.zeros((0, 2))
            self._red_jumps = RedJumps(self.cov_red, de, bounds, self.ctx.device)
            self._red_warm_chain = chain
            return x1
        if rind.size == 0:
            return xnew
        eng = self._red_engine(xnew, 1, chain_base=HOST_CHAIN)
        eng.b[0, :len(self._b)] = torch.as_tensor(self._b, device=self.ctx.device)
        eng.it = self._ndraw
        eng._tau()
        eng.red_block(RED_STEPS)
        self._ndraw += 1
        return eng.x[0].cpu().numpy()

    # ------------------------------------------------------------ loop
    def _red_loop(self):
        if self.red_sig is None:
            return False
        extra = [n for n in self.param_names if "rho" not in n]
        return bool(extra) and all(("log10_A" in n or "gamma" in n) for n in extra)

    def _white_loop(self):
        names = self.param_names
        extra = [n for n in names if "rho" not in n]
        return bool(extra) and all(("efac" in n or "equad" in n) for n in extra)

    def _check_device_loop(self, xs):
        if (self._red_loop() or self._ecorr_loop()) and self.hypersample == "conditional":
            return
        extra = [n for n in self.param_names if "rho" not in n and not self._white_loop()]
        if extra or self.red_sig is not None or self.hypersample != "conditional":
            raise NotImplementedError(
                "the device sweep covers free-spectrum-only models (analytic rho|b); "
                f"found Metropolis-sampled parameters {extra[:4]}...")
        gwind = self.get_gwrho_param_indices()
        if not self._white_loop() and not np.array_equal(gwind, np.arange(len(self.gwid) // 2)):
            raise NotImplementedError("gw rho parameters must be the whole parameter vector")

    def sample(self, xs, outdir="./", niter=10000, resume=False, save_every=100, *, flush_final=False,
               record_bchains=None):
        """PulsarBlockGibbs.sample (pulsar_gibbs.py:620-710) as persistent device sweeps.

        Chain row ii holds the state BEFORE sweep ii (row 0 = xs, bchain[0] = 0).
        Files: pars_chain.txt, pars_bchain.txt, chain.npy, bchain.npy (chain 0,
        rows [:ii+1] written at ii % 100 == 0, ii > 0, as the reference), and with
        nchains > 1 also chains.npy / bchains.npy (leading chain axis)."""
        self._check_device_loop(xs)
        print(f"Creating chain directory: {outdir}")
        os.makedirs(outdir, exist_ok=True)
        np.savetxt(f"{outdir}/pars_chain.txt", self.param_names, fmt="%s")
        np.savetxt(f"{outdir}/pars_bchain.txt", self.b_param_names, fmt="%s")

        if self._red_loop():
            out = self._sample_red(xs, outdir, niter, resume, save_every)
            if flush_final:
                self._flush(outdir)
            return out
        if self._ecorr_loop():
            out = self._sample_ecorr(xs, outdir, niter, resume, save_every)
            if flush_final:
                self._flush(outdir)
            return out
        if self._white_loop():
            out = self._sample_white(xs, outdir, niter, resume, save_every)
            if flush_final:
                self._flush(outdir)
            return out
        sample_free_spectrum([self], self._model(xs), [xs], [outdir], niter, resume, save_every,
                             record_bchains=record_bchains)
        if flush_final:
            self._flush(outdir)
        return self.chain

    def _flush(self, outdir):
        """flush_final=True: also write the rows after the last multiple of
        save_every, which the reference never saves (pulsar_gibbs.py:701-710, Appendix A.8)."""
        save_rows(self, outdir, self.iter + 1, self.chains is not None,
                  getattr(self, "bchains", None) is not None)

    def _sample_white(self, xs, outdir, niter, resume, save_every):
        """sample() with the white-noise MH block (pulsar_gibbs.py:656-698): one device
        launch sequence per sweep for all chains (white.WhiteFreeSpectrumChains)."""
        nc = self.nchains
        dev = self.ctx.device
        wm = self._white_model(xs, nc)
        m = int(wm.m[0])
        n_param = len(xs)
        self.chain = np.zeros((niter, n_param))
        self.bchain = np.zeros((niter, len(self._b)))
        self.chains = np.zeros((nc, niter, n_param)) if nc > 1 else None
        self.bchains = np.zeros((nc, niter, len(self._b))) if nc > 1 else None
        start = 0
        x0 = np.asarray(xs, float)
        acl = getattr(self, "aclength_white", None)
        if resume and os.path.exists(f"{outdir}/chain.npy"):
            print("Resuming from previous run...")
            c0 = np.load(f"{outdir}/chain.npy")
            b0 = np.load(f"{outdir}/bchain.npy")
            start = min(c0.shape[0], b0.shape[0])
            self.chain[:start] = c0[:start]
            self.bchain[:start] = b0[:start]
        runner = WhiteFreeSpectrumChains(wm, n_param, self.get_gwrho_param_indices(), self.rhomin,
                                         self.rhomax, x0, aclength=acl)
        if start > 0:
            runner.x.copy_(torch.as_tensor(self.chain[start - 1][None, :], device=dev).expand(nc, -1))
            runner.b[:, :m] = torch.as_tensor(self.bchain[start - 1], device=dev)
            runner.it = start
            if runner.aclength is None:
                raise NotImplementedError("resume of a white-noise run needs aclength_white")
        blk = max(1, save_every)
        xr = torch.empty(blk + 1, nc, n_param, dtype=torch.float64, device=dev)
        br = torch.empty(blk + 1, nc, wm.ldb, dtype=torch.float64, device=dev)
        ii = start
        while ii < niter:
            nxt = min(niter, (ii // blk + 1) * blk + 1)
            n = nxt - ii
            for k in range(n):
                runner.sweep(x_rec=xr[k], b_rec=br[k])
            xh = xr[:n].cpu().numpy()
            bh = br[:n, :, :m].cpu().numpy()
            self.chain[ii:nxt] = xh[:, 0]
            self.bchain[ii:nxt] = bh[:, 0]
            if nc > 1:
                self.chains[:, ii:nxt] = np.moveaxis(xh, 1, 0)
                self.bchains[:, ii:nxt] = np.moveaxis(bh, 1, 0)
            ii = nxt
            self.iter = ii - 1
            last = ii - 1
            if last % save_every == 0 and last > 0:
                save_rows(self, outdir, last + 1, nc > 1, nc > 1)
        if runner.short_chain is not None:
            sc = runner.short_chain
            self.cov_white = np.cov(sc[100:, :], rowvar=False)
            self.sigma_white = np.diag(np.atleast_2d(self.cov_white)) ** 0.5
            self.svd_white = np.linalg.svd(np.atleast_2d(self.cov_white))
        acl = np.atleast_1d(runner.aclength)
        self.aclength_white = int(acl[0])
        self.aclength_white_chains = acl
        info = runner.info.cpu().numpy()
        if info.any():
            print(f"WARNING: {int((info != 0).sum())} chains hit a non-positive-definite Sigma")
        self._b = runner.b[0, :m].cpu().numpy()
        self._runner = runner
        return self.chain

    def _sample_ecorr(self, xs, outdir, niter, resume, save_every):
        """sample() with the basis-ECORR MH block in the notebook sampler's order (ECORR
        block, rho|b, gated b; pulsar_gibbs.py:656-698 with :675-683 enabled): one device
        launch sequence per sweep for all chains (ecorr.EcorrFreeSpectrumChains)."""
        nc = self.nchains
        dev = self.ctx.device
        white = self._ecorr_white()
        em = self._ecorr_model(xs, nc, per_chain=white)
        m, n_param = em.m, len(xs)
        self.chain = np.zeros((niter, n_param))
        self.bchain = np.zeros((niter, len(self._b)))
        self.chains = np.zeros((nc, niter, n_param)) if nc > 1 else None
        self.bchains = np.zeros((nc, niter, len(self._b))) if nc > 1 else None
        start = 0
        x0 = np.asarray(xs, float)
        if resume and os.path.exists(f"{outdir}/chain.npy"):
            print("Resuming from previous run...")
            c0 = np.load(f"{outdir}/chain.npy")
            b0 = np.load(f"{outdir}/bchain.npy")
            start = min(c0.shape[0], b0.shape[0])
            self.chain[:start] = c0[:start]
            self.bchain[:start] = b0[:start]
        if white:
            # both warm-ups (update_white_params / update_ecorr_params iters=1000, notebook
            # sample() at ii == 0) run once on the 1-chain device models from xs to set the
            # step counts; every chain then starts from their final state
            if getattr(self, "aclength_white", None) is None or getattr(self, "aclength_ecorr", None) is None:
                if not np.any(self._b):
                    self._b = self.update_b(x0)
                x0 = self.update_white_params(x0, iters=1000)
                x0 = self.update_ecorr_params(x0, iters=1000)
            runner = EcorrWhiteChains(self._white_model(xs, nc), em, self.get_gwrho_param_indices(), self.gwid,
                                      self.rhomin, self.rhomax, x0, self.aclength_white, self.aclength_ecorr,
                                      wmR=self._white_model(xs, nc, cols=em.rc_host))
            runner.aclength = self.aclength_ecorr
            runner.short_chain = None
        else:
            runner = EcorrFreeSpectrumChains(em, self.get_gwrho_param_indices(), self.gwid, self.rhomin,
                                             self.rhomax, x0, aclength=getattr(self, "aclength_ecorr", None))
        if start > 0:
            if runner.aclength is None:
                raise NotImplementedError("resume of an ECORR run needs aclength_ecorr")
            runner.x.copy_(torch.as_tensor(self.chain[start - 1][None, :], device=dev).expand(nc, -1))
            runner.b[:, :m] = torch.as_tensor(self.bchain[start - 1], device=dev)
            runner.it = start
        blk = max(1, save_every)
        xr = torch.empty(blk + 1, nc, n_param, dtype=torch.float64, device=dev)
        br = torch.empty(blk + 1, nc, m, dtype=torch.float64, device=dev)
        ii = start
        while ii < niter:
            nxt = min(niter, (ii // blk + 1) * blk + 1)
            n = nxt - ii
            for k in range(n):
                runner.sweep(x_rec=xr[k], b_rec=br[k])
            xh = xr[:n].cpu().numpy()
            bh = br[:n].cpu().numpy()
            self.chain[ii:nxt] = xh[:, 0]
            self.bchain[ii:nxt] = bh[:, 0]
            if nc > 1:
                self.chains[:, ii:nxt] = np.moveaxis(xh, 1, 0)
                self.bchains[:, ii:nxt] = np.moveaxis(bh, 1, 0)
            ii = nxt
            self.iter = ii - 1
            last = ii - 1
            if last % save_every == 0 and last > 0:
                save_rows(self, outdir, last + 1, nc > 1, nc > 1)
        if runner.short_chain is not None:
            sc = runner.short_chain
            self.cov_ecorr = np.cov(sc[100:, :], rowvar=False)
            self.sigma_ecorr = np.diag(np.atleast_2d(self.cov_ecorr)) ** 0.5
            self.svd_ecorr = np.linalg.svd(np.atleast_2d(self.cov_ecorr))
        self.aclength_ecorr = runner.aclength
        if int(em.binfo.max()) != 0:
            print("WARNING: chains hit a non-positive-definite Sigma")
        self._b = runner.b[0, :m].cpu().numpy()
        self._runner = runner
        return self.chain

    def _sample_red(self, xs, outdir, niter, resume, save_every):
        """sample() with power-law red noise (pulsar_gibbs.py:656-698): sweep 0 runs the
        warm-up (update_red_params(iters=10000), :689-690) on the host with the device
        likelihood; every sweep is then one launch sequence for all chains
        (rednoise.RedNoiseChains)."""
        nc = self.nchains
        dev = self.ctx.device
        n_param = len(xs)
        model = self._model(xs)
        m = int(model.m[0])
        self.chain = np.zeros((niter, n_param))
        self.bchain = np.zeros((niter, len(self._b)))
        self.chains = np.zeros((nc, niter, n_param)) if nc > 1 else None
        self.bchains = np.zeros((nc, niter, len(self._b))) if nc > 1 else None
        start = 0
        x0 = np.asarray(xs, float)
        if resume and os.path.exists(f"{outdir}/chain.npy"):
            print("Resuming from previous run...")
            c0 = np.load(f"{outdir}/chain.npy")
            b0 = np.load(f"{outdir}/bchain.npy")
            start = min(c0.shape[0], b0.shape[0])
            self.chain[:start] = c0[:start]
            self.bchain[:start] = b0[:start]
        x_first = None
        if start == 0 and getattr(self, "_red_jumps", None) is None:
            x_first = self.update_red_params(x0, iters=getattr(self, "red_warmup_iters", 10000))
        elif getattr(self, "_red_jumps", None) is None:
            raise NotImplementedError("resume of a red-noise run needs the warm-up's proposal (_red_jumps)")
        runner = self._red_engine(x0, nc, x_first=x_first)
        if start > 0:
            runner.x.copy_(torch.as_tensor(self.chain[start - 1][None, :], device=dev).expand(nc, -1))
            runner.b[:, :m] = torch.as_tensor(self.bchain[start - 1], device=dev)
            runner.it = start
        blk = max(1, save_every)
        xr = torch.empty(blk + 1, nc, n_param, dtype=torch.float64, device=dev)
        br = torch.empty(blk + 1, nc, model.ldb, dtype=torch.float64, device=dev)
        ii = start
        while ii < niter:
            nxt = min(niter, (ii // blk + 1) * blk + 1)
            n = nxt - ii
            for k in range(n):
                runner.sweep(x_rec=xr[k], b_rec=br[k])
            xh = xr[:n].cpu().numpy()
            bh = br[:n, :, :m].cpu().numpy()
            self.chain[ii:nxt] = xh[:, 0]
            self.bchain[ii:nxt] = bh[:, 0]
            if nc > 1:
                self.chains[:, ii:nxt] = np.moveaxis(xh, 1, 0)
                self.bchains[:, ii:nxt] = np.moveaxis(bh, 1, 0)
            ii = nxt
            self.iter = ii - 1
            last = ii - 1
            if last % save_every == 0 and last > 0:
                save_rows(self, outdir, last + 1, nc > 1, nc > 1)
        info = runner.info.cpu().numpy()
        if info.any():
            print(f"WARNING: {int((info != 0).sum())} chains hit a non-positive-definite Sigma")
        steps = runner.n_blocks * runner.nsteps
        self.red_acceptance = (runner.acc_total.cpu().numpy() / steps) if steps else None
        self._b = runner.b[0, :m].cpu().numpy()
        self._runner = runner
        return self.chain
