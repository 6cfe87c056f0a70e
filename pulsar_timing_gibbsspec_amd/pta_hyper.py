"""PTA red-noise hyper-parameters by Metropolis (``PTABlockGibbs(redsample='mh')``, the
reference's default; SURVEY §8f-2, PTA half).

Reference: ``PTABlockGibbs.update_hyper_params`` pta_gibbs.py:278-340 with the summed
marginalised likelihood ``get_lnlikelihood`` :577-621 and the sweep order :689-697.  Each
sweep runs ``aclength_hyper`` single-parameter Metropolis steps over the red parameters
``hind`` (every pulsar's power-law ``log10_A``/``gamma`` or red free-spectrum ``rho``):
scale from ``choice(sizes, p=probs)``, one parameter by ``choice(hind)``, q[par] += randn *
(0.05 len(hind)) * scale, accept if (lnL(q) + lnprior(q)) - (lnL(x) + lnprior(x)) > log(rand).

Here the block is one kernel per sweep for every chain (``gs_hyper_mh``): a step moves one
pulsar's parameter, so only that pulsar's marginalised likelihood is re-evaluated (the
other 44 terms and the uniform prior constants cancel in the difference), seeded each
block by ``gs_lnlike_marg`` over all (pulsar, chain) systems.  Out-of-prior proposals are
rejected without a likelihood (the reference evaluates them first, and the overflowed
power-law phi of a far proposal kills its cho_factor).

Sweep 0 (``iters=100``, :283-315): the reference computes cov / SVD / acor of
``short_chain[100:]`` -- empty for its own 100 steps, so numpy's SVD of the NaN covariance
raises LinAlgError and the reference's default path cannot pass sweep 0.  Here the 100
warm-up steps run as in the reference and ``aclength_hyper`` (unless the caller set it)
is the acor restatement (diagnostics.acor) over the whole warm-up proposal chain of chain 0.
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib
from ._lib import check, ptr
from .diagnostics import acor
from .engine import _t
from .plumbing import expand_names, uniform_bounds, vector_to_dict
from .rednoise import powerlaw_loglinear

HYPER_WARMUP = 100      # update_hyper_params(xnew, iters=100) at sweep 0 (pta_gibbs.py:694-695)
RED_FREESPEC, RED_POWERLAW = 0, 1


def hyper_aclength(short_chain, burn=100):
    """aclength_hyper = max_j int(acor(short_chain[burn:, j])[0]) (pta_gibbs.py:314-315), over
    the whole warm-up when the reference's slice is empty (its own iters=100), at least 1."""
    sc = np.asarray(short_chain, float)
    if sc.shape[0] > burn:
        sc = sc[burn:]
    return max(1, int(np.max([int(acor(sc[:, j])[0]) for j in range(sc.shape[1])])))


class HyperSpec:
    """Device tables of the red hyper-parameters of a PTA (pta_gibbs.py:156-162 indices):
    hcol = hind (x columns), hpsr = owning pulsar, uniform prior box, and per pulsar either the
    free-spectrum columns (red_col [P x n_f]) or the power-law (log10_A, gamma) columns
    (pl_col [P x 2]) with the log-linear phi table lnphi [P x 3 x n_f] probed from the signal's
    own get_phi."""

    def __init__(self, pta, params, red_sigs, hind, x_ref, n_f, device):
        names = expand_names(params)
        col_of = {n: i for i, n in enumerate(names)}
        by_name = {p.name: p for p in params}
        P = len(pta.pulsars)
        if len(red_sigs) != P:
            raise NotImplementedError(f"redsample='mh' needs one red signal per pulsar ({len(red_sigs)} for {P})")
        hind = np.asarray(hind, np.int64)
        owner = np.full(len(names), -1, np.int64)
        kinds, red_col, pl_col, lnphi = [], np.zeros((P, n_f), np.int32), np.zeros((P, 2), np.int32), []
        base = vector_to_dict(params, np.asarray(x_ref, float))
        for p, sig in enumerate(red_sigs):
            sp = list(sig.params)
            cols = [col_of[n] for n in expand_names(sp)]
            owner[cols] = p
            pn = [q.name for q in sp]
            la = [q for q in sp if "log10_A" in q.name]
            ga = [q for q in sp if "gamma" in q.name]
            if len(sp) == 1 and "rho" in pn[0] and (sp[0].size or 1) == n_f:
                kinds.append(RED_FREESPEC)
                red_col[p] = cols
            elif len(sp) == 2 and len(la) == 1 and len(ga) == 1:
                kinds.append(RED_POWERLAW)
                pl_col[p] = [col_of[la[0].name], col_of[ga[0].name]]

                def phi_of(a, g, sig=sig, la=la[0].name, ga=ga[0].name):
                    prm = dict(base)
                    prm[la], prm[ga] = a, g
                    return np.asarray(sig.get_phi(prm), float)[::2]
                lnphi.append(powerlaw_loglinear(phi_of))
            else:
                raise NotImplementedError(f"red signal {sig.name!r} of pulsar {p}: params {pn} are neither a "
                                          f"{n_f}-bin free spectrum nor a (log10_A, gamma) power law")
        if len(set(kinds)) != 1:
            raise NotImplementedError("mixed red-noise models across pulsars")
        self.kind = kinds[0]
        if (owner[hind] < 0).any():
            raise NotImplementedError("a red hyper-parameter belongs to no pulsar's red signal")
        bounds = []
        for n in np.asarray(names)[hind]:
            base_name = n if n in by_name else n.rsplit("_", 1)[0]
            bounds.append(uniform_bounds(by_name[base_name]))
        bounds = np.asarray(bounds, float)
        self.P, self.n_f, self.n_h = P, n_f, hind.size
        self.hind = hind
        self.hpsr_host = owner[hind]
        self.hlo_host, self.hhi_host = bounds[:, 0], bounds[:, 1]
        self.red_col_host, self.pl_col_host = red_col, pl_col
        self.lnphi_host = np.stack(lnphi) if lnphi else np.zeros((P, 3, n_f))
        self.hcol = _t(hind.astype(np.int32), torch.int32, device)
        self.hpsr = _t(self.hpsr_host.astype(np.int32), torch.int32, device)
        self.hlo = _t(self.hlo_host, torch.float64, device)
        self.hhi = _t(self.hhi_host, torch.float64, device)
        self.red_col = _t(red_col.ravel(), torch.int32, device)
        self.pl_col = _t(pl_col.ravel(), torch.int32, device)
        self.lnphi = _t(self.lnphi_host.ravel(), torch.float64, device)

    def short_chain(self, x_start, q_rec):
        """The reference's short_chain rows q[hind] (pta_gibbs.py:309) of one chain from its
        hind values at the block start and the kernel's (j, proposal, accepted) records."""
        cur = np.asarray(x_start, float)[self.hind].copy()
        rows = np.empty((len(q_rec), self.n_h))
        for s, (j, q, acc) in enumerate(q_rec):
            j = int(j)
            rows[s] = cur
            rows[s, j] = q
            if acc:
                cur[j] = q
        return rows


class HyperMH:
    """The device side of one PTA engine's hyper block: per-(pulsar, chain) lnL_p and the
    launches (seed lnL_p from the phiinv of the current x, then gs_hyper_mh)."""

    def __init__(self, spec: HyperSpec, model, n_chain, n_param, gw_col, psr_lo=0):
        """psr_lo: the model holds pulsars [psr_lo, psr_lo + model.P) of the spec's array (a
        pulsar-sharded rank).  The step tables are then this rank's: a parameter of another rank's
        pulsar gets hpsr = -1 and its steps are skipped (every rank draws the same step table from
        the chain-level Philox counters, and each applies the steps of its own pulsars -- each
        pulsar's subsequence in the reference's order; pta_gibbs.py:294-305), and the per-pulsar
        tables (red columns, power-law table) are the model's slices.  The red phi of every pulsar
        (``irn``, for the common draw) uses the spec's whole-array tables."""
        self.spec, self.model, self.ctx = spec, model, model.ctx
        self.C, self.n_param = int(n_chain), int(n_param)
        dev = self.ctx.device
        self.gw_col = gw_col
        lo, P = int(psr_lo), model.P
        if lo < 0 or lo + P > spec.P:
            raise ValueError(f"pulsars [{lo}, {lo + P}) outside the spec's {spec.P}")
        hp = spec.hpsr_host - lo
        hp[(hp < 0) | (hp >= P)] = -1
        self.hpsr = _t(hp.astype(np.int32), torch.int32, dev)
        self.red_col = _t(spec.red_col_host[lo:lo + P].ravel(), torch.int32, dev)
        self.pl_col = _t(spec.pl_col_host[lo:lo + P].ravel(), torch.int32, dev)
        self.lnphi = _t(spec.lnphi_host[lo:lo + P].ravel(), torch.float64, dev)
        self.lnl_p = torch.empty(model.P * self.C, dtype=torch.float64, device=dev)
        self.n_acc = torch.zeros(self.C, dtype=torch.int32, device=dev)
        self.acc_total = torch.zeros(self.C, dtype=torch.int64, device=dev)
        self.steps_total = 0
        self.fresh = False      # lnl_p holds lnL_p at the current x (set by the engine's b draw)

    def seed(self, phiinv_F):
        """lnl_p[p * C + c] = phi-dependent lnL of system (p, c) at the phiinv rows given."""
        m = self.model
        check(self.ctx.lib.gs_lnlike_marg(self.ctx.handle, m.P, self.C, m.NF, m.NMX, ptr(m.model), 0,
                                          ptr(m.nm_dev), ptr(phiinv_F), ptr(self.lnl_p), None), "gs_lnlike_marg")

    def steps(self, x, nsteps, sweep, chain_base, inj=None, q_rec=None):
        m, sp = self.model, self.spec
        if nsteps <= 0:
            return
        if inj is not None:
            if tuple(inj.shape) != (int(nsteps), self.C, 4):
                raise ValueError(f"inj must be (nsteps, n_chain, 4) = {(int(nsteps), self.C, 4)}, got "
                                 f"{tuple(inj.shape)}")
            j = inj[..., 1]
            # a host check of a device tensor syncs (and raises inside graph capture): validated on
            # CPU tensors and outside capture only -- the kernel clamps j either way
            chk = inj.device.type == "cpu" or not torch.cuda.is_current_stream_capturing()
            if chk and bool(((j < 0) | (j > sp.n_h - 1) | (j != torch.floor(j))).any()):
                raise ValueError(f"inj[..., 1] (the parameter index) must be an integer in [0, {sp.n_h - 1}]")
        check(self.ctx.lib.gs_hyper_mh(self.ctx.handle, m.P, self.C, m.NF, m.NMX, ptr(m.model), ptr(m.nm_dev),
                                       ptr(x), self.n_param, ptr(self.gw_col), sp.n_h, ptr(sp.hcol), ptr(self.hpsr),
                                       ptr(sp.hlo), ptr(sp.hhi), sp.kind, ptr(self.red_col), ptr(self.pl_col),
                                       ptr(self.lnphi), ptr(self.lnl_p), int(nsteps), int(sweep), int(chain_base),
                                       ptr(inj), ptr(q_rec), ptr(self.n_acc)), "gs_hyper_mh")
        self.acc_total += self.n_acc
        self.steps_total += int(nsteps)

    def irn(self, x, out):
        """Per-pulsar red phi [P x n_f x C] of the whole array at x (power law; the free spectrum uses
        gs_phi_from_x)."""
        sp = self.spec
        check(self.ctx.lib.gs_phi_powerlaw(self.ctx.handle, sp.P, self.C, sp.n_f, ptr(x), self.n_param,
                                           ptr(sp.pl_col), ptr(sp.lnphi), ptr(out)), "gs_phi_powerlaw")

    def acceptance(self):
        return (self.acc_total.double() / max(1, self.steps_total)).cpu().numpy()


def mh_injection(kinds, vals, lens, hind, start, nsteps):
    """(scale, j, randn, rand) rows of ``nsteps`` MH steps from a captured draw log, starting at
    entry ``start`` (4 entries per step: choice, choice, randn, rand).  Returns (rows, next)."""
    offs = np.concatenate([[0], np.cumsum(lens)])
    pos = {int(h): j for j, h in enumerate(hind)}
    rows = np.empty((nsteps, 4))
    k = start
    for s in range(nsteps):
        assert tuple(kinds[k:k + 4]) == ("choice", "choice", "randn", "rand"), (k, kinds[k:k + 4])
        v = [vals[offs[k + i]:offs[k + i + 1]] for i in range(4)]
        rows[s] = [v[0][0], pos[int(v[1][0])], v[2][0], v[3][0]]
        k += 4
    return rows, k
