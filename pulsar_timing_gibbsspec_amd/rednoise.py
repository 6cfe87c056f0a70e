"""Power-law intrinsic red noise on the device.

The reference samples a power-law red process (log10_A, gamma) next to the free
spectrum with PTMCMCSampler (``PulsarBlockGibbs.update_red_params``
pulsar_gibbs.py:271-329): a 10,000-step warm-up on the full marginalised likelihood
at sweep 0 (:283-309) learns the proposal covariance, then every sweep runs 20
``PTMCMCOneStep`` calls on the red-only likelihood ``get_lnlikelihood_red``
(:549-566, :312-319), and rho|b switches to the grid + Gumbel-max draw (:218-234).

Here the per-sweep block is one kernel for all chains (``gs_red_mh``), the Gumbel draw
is ``gs_rho_gumbel`` and the gated b-draw takes phi = 10^(2 rho) + irn
(``gs_gate_phiinv_irn``).  The warm-up runs on the host with the device's marginalised
likelihood (``gs_lnlike_marg``) and restates PTMCMCSampler's adaptive SCAM/AM jumps;
PTMCMCSampler itself is absent (no pinned version), so the proposal law is a
restatement ("parity unpinned" for the jumps) while the
likelihood, the acceptance semantics and the sweep order follow the reference.
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib
from ._lib import check, ptr
from .engine import DeviceModel, _t, grid3

# PTMCMCSampler weights of the reference's warm-up call (pulsar_gibbs.py:295-296)
W_SCAM, W_AM, W_DE = 30.0, 15.0, 50.0
RED_STEPS = 20          # step_max (pulsar_gibbs.py:316)
COV_UPDATE = 1000       # PTMCMCSampler's covariance update period
DE_BUFFER = 1000


def powerlaw_loglinear(phi_of, la_probe=(0.0, -20.0), ga_probe=(0.0, 7.0), check_at=(-14.3, 3.7)):
    """log phi_red(f_k) = c_k + a_k log10_A + g_k gamma for a power-law PSD.

    ``phi_of(log10_A, gamma)`` returns the red phi at the sin columns (the reference's
    ``red_sig.get_phi(params)[::2]``).  Slopes come from widely separated probes; the
    form is verified at ``check_at`` (NotImplementedError for a non-power-law PSD)."""
    l00 = np.log(phi_of(la_probe[0], ga_probe[0]))
    a = (l00 - np.log(phi_of(la_probe[1], ga_probe[0]))) / (la_probe[0] - la_probe[1])
    g = (np.log(phi_of(la_probe[0], ga_probe[1])) - l00) / (ga_probe[1] - ga_probe[0])
    c = l00 - a * la_probe[0] - g * ga_probe[0]
    lnphi = np.stack([c, a, g])
    want = np.log(phi_of(*check_at))
    got = (a * check_at[0] + c) + g * check_at[1]
    if not np.allclose(got, want, rtol=1e-11, atol=1e-11):
        raise NotImplementedError("the red-noise PSD is not a power law in (log10_A, gamma)")
    return lnphi


def jump_table(cov, bounds, nde):
    """gs_red_mh's jump[12]: SVD of the 2x2 proposal covariance, cumulative SCAM / AM
    probabilities (DE gets the rest, only with a buffer of >= 2 samples), prior bounds."""
    U, S, _ = np.linalg.svd(np.asarray(cov, float))
    tot = W_SCAM + W_AM + (W_DE if nde >= 2 else 0.0)
    return np.array([U[0, 0], U[0, 1], U[1, 0], U[1, 1], np.sqrt(S[0]), np.sqrt(S[1]),
                     W_SCAM / tot, (W_SCAM + W_AM) / tot,
                     bounds[0][0], bounds[0][1], bounds[1][0], bounds[1][1]])


class RedJumps:
    """Proposal state learnt by the warm-up: red-block covariance (log10_A, gamma order)
    and the DE buffer of warm-up samples."""

    def __init__(self, cov, de, bounds, device):
        self.cov = np.asarray(cov, float)
        self.de_host = np.ascontiguousarray(np.asarray(de, float).reshape(-1, 2))
        self.nde = len(self.de_host)
        self.table_host = jump_table(self.cov, bounds, self.nde)
        self.table = _t(self.table_host, torch.float64, device)
        self.de = _t(self.de_host if self.nde else np.zeros((1, 2)), torch.float64, device)


def warmup(lnprob, x0, iters, rng, bounds_lo, bounds_hi, cov0=0.01):
    """The sweep-0 warm-up (pulsar_gibbs.py:283-309) restated: an adaptive Metropolis run
    of ``iters`` steps over every parameter from x0 (PTMCMCSampler.sample with SCAM 30 /
    AM 15 jumps, cov = 0.01 I adapted every 1000 steps from the chain so far; DE needs a
    buffer PTMCMCSampler fills only after ``burn = iters - 1``, so it never fires here),
    followed by ONE joint step from x0 with the adapted covariance (:298: the warm-up's
    own end state is discarded).  lnprob(x) -> float.  Returns (x1, cov, chain)."""
    x0 = np.asarray(x0, float)
    nd = x0.size
    cov = cov0 * np.eye(nd)
    U, S, _ = np.linalg.svd(cov)

    def propose(x):
        u = rng.random()
        scale = 10.0 if u > 0.97 else (0.2 if u > 0.9 else 1.0)
        q = x.copy()
        if rng.random() < W_SCAM / (W_SCAM + W_AM):
            j = rng.integers(nd)
            q += rng.standard_normal() * 2.4 / np.sqrt(2.0) * scale * np.sqrt(S[j]) * U[:, j]
        else:
            q += 2.4 / np.sqrt(2.0 * nd) * scale * (U @ (rng.standard_normal(nd) * np.sqrt(S)))
        return q

    def inb(q):
        return bool(np.all(q >= bounds_lo) and np.all(q <= bounds_hi))

    x, lp = x0.copy(), lnprob(x0)
    chain = np.empty((max(iters - 1, 0), nd))
    for i in range(iters - 1):
        q = propose(x)
        lq = lnprob(q) if inb(q) else -np.inf
        if lq - lp > np.log(rng.random()):
            x, lp = q, lq
        chain[i] = x
        if (i + 1) % COV_UPDATE == 0:
            cov = np.cov(chain[:i + 1], rowvar=False) + 1e-12 * np.eye(nd)
            U, S, _ = np.linalg.svd(cov)
    q = propose(x0)                                   # PTMCMCOneStep(xnew, ...) from x0
    lq = lnprob(q) if inb(q) else -np.inf
    x1 = q if lq - lnprob(x0) > np.log(rng.random()) else x0.copy()
    return x1, cov, chain


class RedNoiseChains:
    """n_chain chains of the single-pulsar free spectrum + power-law red noise model
    (PulsarBlockGibbs.sample with a red signal, pulsar_gibbs.py:656-698):

      record x, b -> [ii == 0: b|rho from x0] -> tau (half) -> red MH block (gs_red_mh,
      20 steps) -> gw rho|b grid + Gumbel (gs_rho_gumbel, irn from the new red state)
      -> gate + phiinv (phi = 10^(2 rho) + irn) -> gated b|rho.

    ``x_first`` (n_chain, n_param), optional: the state after sweep 0's red block (the
    warm-up's joint step), used instead of the 20-step block at sweep 0."""

    def __init__(self, model: DeviceModel, n_param, gw_col, red_col, lnphi, jumps: RedJumps, rhomin, rhomax,
                 n_chain, x0, chain_base=0, nsteps=RED_STEPS, anchor=1, ngrid=1000, x_first=None):
        if model.P != 1:
            raise ValueError("RedNoiseChains models one pulsar")
        self.model, self.ctx = model, model.ctx
        dev = self.ctx.device
        C = int(n_chain)
        self.C, self.n_param, self.n_f = C, int(n_param), model.NF // 2
        self.chain_base, self.nsteps, self.anchor, self.ngrid = int(chain_base), int(nsteps), int(anchor), ngrid
        self.gw_col = _t(np.asarray(gw_col, np.int32), torch.int32, dev)
        self.red_col = _t(np.asarray(red_col, np.int32), torch.int32, dev)
        self.lnphi = _t(np.asarray(lnphi, float), torch.float64, dev)
        self.jumps = jumps
        self.grid = grid3(rhomin, rhomax, n=ngrid, device=dev)
        self.x = _t(np.broadcast_to(np.asarray(x0, float), (C, self.n_param)), torch.float64, dev)
        self.x_first = None if x_first is None else _t(np.broadcast_to(np.asarray(x_first, float),
                                                                       (C, self.n_param)), torch.float64, dev)
        self.b = torch.zeros(C, model.ldb, dtype=torch.float64, device=dev)
        self.tau = torch.empty(self.n_f, C, dtype=torch.float64, device=dev)
        self.irn = torch.empty(self.n_f, C, dtype=torch.float64, device=dev)
        self.lnl = torch.empty(C, dtype=torch.float64, device=dev)
        self.n_acc = torch.zeros(C, dtype=torch.int32, device=dev)
        self.acc_total = torch.zeros(C, dtype=torch.int64, device=dev)
        self.n_blocks = 0
        self.phiinv_F = torch.empty(C, model.NF, dtype=torch.float64, device=dev)
        self.gate = torch.ones(C, dtype=torch.int32, device=dev)
        self.xlast = torch.empty(C, dtype=torch.float64, device=dev)
        self.info = torch.zeros(C, dtype=torch.int32, device=dev)
        self.it = 0

    # ------------------------------------------------------------------ pieces
    def _tau(self):
        m = self.model
        check(self.ctx.lib.gs_tau(self.ctx.handle, 1, self.C, m.NF, m.ldb, ptr(m.fidx), ptr(self.b), 1,
                                  ptr(self.tau)), "gs_tau")

    def red_block(self, nsteps):
        """gs_red_mh over every chain with the current b (tau) and x; nsteps = 0 only
        evaluates lnL / irn at the current state."""
        j = self.jumps
        check(self.ctx.lib.gs_red_mh(self.ctx.handle, self.C, self.n_f, int(nsteps), self.anchor, ptr(self.x),
                                     self.n_param, ptr(self.red_col), ptr(self.gw_col), ptr(self.tau),
                                     ptr(self.lnphi), ptr(j.table), ptr(j.de), j.nde, self.it,
                                     self.chain_base, ptr(self.irn), ptr(self.lnl), ptr(self.n_acc)),
              "gs_red_mh")

    def _gate_phiinv(self, with_gate):
        check(self.ctx.lib.gs_gate_phiinv_irn(self.ctx.handle, self.C, self.n_f, self.n_param, ptr(self.x),
                                              ptr(self.xlast) if with_gate else None, ptr(self.gw_col),
                                              ptr(self.irn), ptr(self.phiinv_F), ptr(self.gate)),
              "gs_gate_phiinv_irn")

    def _bdraw(self, event, mask, z=None):
        self.model.bdraw(self.phiinv_F, self.C, z=z, sweep=self.it, event=event, chain_base=self.chain_base,
                         out=self.b, info=self.info, chain_mask=mask)

    def lnlike_red(self):
        """get_lnlikelihood_red of every chain's current (x, b)."""
        self._tau()
        self.red_block(0)
        return self.lnl

    # ------------------------------------------------------------------ sweep
    def sweep(self, x_rec=None, b_rec=None, u_gumbel=None, z0=None, z=None):
        lib, h = self.ctx.lib, self.ctx.handle
        check(lib.gs_pta_record(h, self.C, self.n_param, ptr(self.x), ptr(x_rec), ptr(self.xlast)),
              "gs_pta_record")                                        # :658-659
        if b_rec is not None:
            b_rec.copy_(self.b)
        if self.it == 0:                                              # :661-662
            self._tau()
            self.red_block(0)
            self._gate_phiinv(with_gate=False)
            self._bdraw(_lib.EV_B0, None, z0)
        self._tau()
        if self.it == 0 and self.x_first is not None:                 # warm-up's joint step
            self.x.copy_(self.x_first)
            self.red_block(0)
        else:
            self.red_block(self.nsteps)                               # :312-319
            self.acc_total += self.n_acc
            self.n_blocks += 1
        check(lib.gs_rho_gumbel(h, self.C, self.n_f, ptr(self.tau), ptr(self.irn), self.ngrid, ptr(self.grid),
                                ptr(u_gumbel), self.it, self.chain_base, ptr(self.x), self.n_param,
                                ptr(self.gw_col), None), "gs_rho_gumbel")   # :218-236
        self._gate_phiinv(with_gate=True)                             # :697
        self._bdraw(_lib.EV_B, self.gate, z)                          # :698
        self.it += 1
