"""Basis ECORR on the device.

The reference's ECORR block is ``PulsarBlockGibbs.update_ecorr_params``
(pulsar_gibbs.py:409-486): single-parameter Metropolis steps on the per-backend
log10_ecorr values under the marginalised likelihood (``self.get_lnlikelihood``, which
the .py never defines -- its sample loop prints 'ERROR: No ECORR for now...' and skips
the block (:675-683); the working sampler is the notebook's
(pta_gibbs_freespec.ipynb, cell 2: ``get_lnlikelihood`` = the code of
``get_lnlikelihood_fullmarg`` :569-610, sweep order white -> ECORR -> rho|b -> gated b).

Device form (csrc/gibbs_ecorr.hip): the epoch columns E of the ECORR basis have a
diagonal TNT block, so every likelihood evaluation and b draw works on the Schur
complement over the remaining columns R = [timing model | free spectrum]:
``gs_ecorr_schur`` (batched fp64-MFMA SYRK over epochs, all chains) ->
``gs_prefix_sys`` -> ``gs_lnlike_marg`` per Metropolis step, and ``gs_bdraw_sys`` on the
R system + ``gs_ecorr_bdraw_e`` for the epochs per b draw.  White noise is fixed (the
configuration of SURVEY 8f-4's J1713 run: efac/equad from a noise dictionary).
"""
from __future__ import annotations

import ctypes
import os

import numpy as np
import torch

from . import _lib
from ._lib import check, ptr
from .engine import TUNED_NF, _t


def group_epochs(ecid, epoch_backend, n_backend):
    """The ECORR epochs grouped by backend, stable within a backend: (ecid, epoch_backend, eoff) with
    eoff [n_backend + 1] the first epoch of each backend (eoff[-1] = number of epochs).  Each backend's
    epochs are then one contiguous row range of [B | d_E], which the incremental Metropolis step
    (gs_ecorr_lnl_state) re-weights alone; the epoch order is otherwise arbitrary (every result is a
    sum over epochs or is written back by epoch column)."""
    ecid = np.asarray(ecid, np.int64)
    ebk = np.asarray(epoch_backend, np.int64)
    if ecid.shape != ebk.shape:
        raise ValueError("ecid and epoch_backend differ in length")
    if ebk.size and (ebk.min() < 0 or ebk.max() >= n_backend):
        raise ValueError(f"epoch_backend must be in 0..{n_backend - 1}")
    order = np.argsort(ebk, kind="stable")
    ebk = ebk[order]
    return ecid[order], ebk, np.searchsorted(ebk, np.arange(n_backend + 1)).astype(np.int32)


class EcorrModel:
    """One pulsar with a basis-ECORR signal, n_chain chains, fixed white noise.

    T (n_toa x m), Nvec, r: host arrays; ecid: the ECORR epoch columns; epoch_backend[e]:
    backend of each epoch (index into ecol); gwid: the NF free-spectrum columns in
    (sin, cos) order; every other column is a fixed-prior (timing-model) column with
    phiinv_fixed (scalar, or one value per such column in increasing column order).
    ecol / emin / emax: x column and Uniform prior of each backend's
    log10_ecorr (eind order).
    """

    def __init__(self, ctx, T, Nvec, r, ecid, epoch_backend, gwid, ecol, emin, emax, n_param, n_chain,
                 phiinv_fixed=1e-40, per_chain=False):
        self.ctx = ctx
        dev = ctx.device
        lib, h = ctx.lib, ctx.handle
        T = np.ascontiguousarray(T, float)
        n_toa, m = T.shape
        ecid = np.asarray(ecid, np.int64)
        ecid, epoch_backend, eoff = group_epochs(ecid, epoch_backend, len(ecol))
        gwid = np.asarray(gwid, np.int64)
        NF = gwid.size
        if NF not in TUNED_NF:
            raise NotImplementedError(f"ECORR path needs NF in {TUNED_NF}, got {NF}")
        self.m, self.ne, self.NF = m, ecid.size, NF
        self.C = int(n_chain)
        self.n_param = int(n_param)
        rc = np.setdiff1d(np.arange(m), ecid)
        self.mR = mR = rc.size
        self.ldbx = 16 * ((mR + 2 + 14) // 16)
        if self.ldbx > 128:
            raise NotImplementedError(f"ECORR Schur kernel supports mR <= 127 (got {mR})")
        pos = {c: i for i, c in enumerate(rc)}
        fR = np.array([pos[c] for c in gwid], np.int32)
        mR_idx = np.array([i for i, c in enumerate(rc) if c not in set(gwid.tolist())], np.int32)
        self.nm = mR - NF
        if not 0 < self.nm <= 64:
            raise NotImplementedError("need 1..64 fixed-prior columns")
        self.NMX = self.nm
        self.rc_host, self.ecid_host = rc, ecid
        # TNT / d of the whole basis once (N fixed), then the chain-independent pieces
        tdesc = np.array([[n_toa, m, 0, 0, 0, 0]], np.int64)
        Td, Nd, rd = _t(T.ravel(), torch.float64, dev), _t(Nvec, torch.float64, dev), _t(r, torch.float64, dev)
        TNT = torch.empty(m * m, dtype=torch.float64, device=dev)
        d = torch.empty(m, dtype=torch.float64, device=dev)
        check(lib.gs_tnt(h, 1, m, ptr(_t(tdesc, torch.int64, dev)), ptr(Td), ptr(Nd), ptr(rd), ptr(TNT), ptr(d)),
              "gs_tnt")
        TNT = TNT.view(m, m)
        e_t = torch.as_tensor(ecid, device=dev)
        r_t = torch.as_tensor(rc, device=dev)
        Bx = torch.zeros(self.ne, self.ldbx, dtype=torch.float64, device=dev)
        Bx[:, :mR] = TNT[e_t][:, r_t]
        Bx[:, mR] = d[e_t]
        self.Bx = Bx.contiguous()
        self.Dg = TNT[e_t, e_t].contiguous()
        self.A = TNT[r_t][:, r_t].contiguous()
        self.dR = d[r_t].contiguous()
        self.TNT_full, self.d_full = TNT, d
        self.ebk = _t(np.asarray(epoch_backend, np.int32), torch.int32, dev)
        self.eoff_host = eoff
        self.eoff = _t(self.eoff_host, torch.int32, dev)
        self.ecol = _t(np.asarray(ecol, np.int32), torch.int32, dev)
        self.ecol_host = np.asarray(ecol, np.int64)
        self.n_bk = len(ecol)
        self.emin = _t(np.asarray(emin, float), torch.float64, dev)
        self.emax = _t(np.asarray(emax, float), torch.float64, dev)
        self.ecid = _t(ecid.astype(np.int32), torch.int32, dev)
        self.rcol = _t(rc.astype(np.int32), torch.int32, dev)
        # R system: prefix over the fixed-prior columns, free spectrum last
        self.fidx = _t(fR[None, :], torch.int32, dev)
        self.midx = _t(mR_idx[None, :], torch.int32, dev)
        self.nm_dev = _t(np.array([self.nm], np.int32), torch.int32, dev)
        phf = np.broadcast_to(np.asarray(phiinv_fixed, float), (self.NMX,))
        self.phfix = _t(phf[None, :], torch.float64, dev)
        self.pdesc = _t(np.array([[mR, self.nm, 0, 0]], np.int64), torch.int64, dev)
        self.mstride = int(lib.gs_model_stride(NF, self.NMX))
        # fused path (gs_ecorr_prefix): columns [M (<= 16) | F | d], phiinv_M on the M diagonal
        self.fused = self.nm <= 16
        self.fused_lnl = True   # likelihood-mode launches for the Metropolis steps
        # Metropolis steps from the stored state (gs_ecorr_lnl_state): only the moved backend's epochs
        # re-weighted per step; a full evaluation starts every block and every REFRESH steps
        self.incremental = os.environ.get("GS_ECORR_INC", "1") != "0"   # (GS_ECORR_INC=0: A/B builds)
        if self.fused:
            KB = 16 * (1 + (NF + 1 + 15) // 16)
            self.ldbp = KB
            mcols = torch.as_tensor(rc[mR_idx], device=dev)
            fcols = torch.as_tensor(gwid, device=dev)
            Bp = torch.zeros(self.ne, KB, dtype=torch.float64, device=dev)
            Bp[:, :self.nm] = TNT[e_t][:, mcols]
            Bp[:, 16:16 + NF] = TNT[e_t][:, fcols]
            Bp[:, 16 + NF] = d[e_t]
            self.Bp = Bp.contiguous()
            cols = torch.cat([mcols, fcols])
            idx = torch.cat([torch.arange(self.nm, device=dev), 16 + torch.arange(NF, device=dev)])
            Ap = torch.zeros(KB, KB, dtype=torch.float64, device=dev)
            Ap[idx[:, None], idx[None, :]] = TNT[cols][:, cols]
            Ap[16 + NF, idx] = d[cols]
            Ap[idx, 16 + NF] = d[cols]
            dm = torch.arange(self.nm, device=dev)
            Ap[dm, dm] += self.phfix[0, :self.nm]
            pad = torch.cat([torch.arange(self.nm, 16, device=dev), torch.arange(17 + NF, KB, device=dev)])
            Ap[pad, pad] = 1.0
            self.Ap = Ap.contiguous()
            # column maps of the reordered layout: original column (-1 pad, -2 d) and R index
            colmap = np.full(KB, -1, np.int32)
            colmap[:self.nm] = rc[mR_idx]
            colmap[16:16 + NF] = gwid
            colmap[16 + NF] = -2
            jmap = np.full(KB, -1, np.int32)
            jmap[:self.nm] = mR_idx
            jmap[16:16 + NF] = fR
            self.colmap = _t(colmap, torch.int32, dev)
            self.jmap = _t(jmap, torch.int32, dev)
            self.dcol = 16 + NF
            phm = np.ones(16)
            phm[:self.nm] = np.asarray(phf)[:self.nm]
            self.phm = _t(phm, torch.float64, dev)
        # per-chain operands (white noise sampled: N, hence TNT, differs per chain)
        self.per_chain = bool(per_chain)
        self.strides = (0, 0, 0)
        if self.per_chain:
            if not self.fused:
                raise NotImplementedError("per-chain ECORR operands need <= 16 fixed-prior columns")
            KB = self.ldbp
            C0 = int(n_chain)
            self.Bp = torch.empty(C0, self.ne, KB, dtype=torch.float64, device=dev)
            self.Dg = torch.empty(C0, self.ne, dtype=torch.float64, device=dev)
            self.Ap = torch.empty(C0, KB, KB, dtype=torch.float64, device=dev)
            self.strides = (self.ne * KB, self.ne, KB * KB)
        C = self.C
        self.TNTc = torch.empty(C * mR * mR, dtype=torch.float64, device=dev)
        self.dc = torch.empty(C * mR, dtype=torch.float64, device=dev)
        self.aux = torch.empty(C, 4, dtype=torch.float64, device=dev)
        self.model = torch.empty(C * self.mstride, dtype=torch.float64, device=dev)
        self.pinfo = torch.zeros(C, dtype=torch.int32, device=dev)
        self.lnl = torch.empty(C, dtype=torch.float64, device=dev)
        self.linfo = torch.zeros(C, dtype=torch.int32, device=dev)
        self._linfo_dirty = False
        self.lnl0 = torch.empty(C, dtype=torch.float64, device=dev)
        self.xq = torch.empty(C, self.n_param, dtype=torch.float64, device=dev)
        self.prop = torch.empty(C, 4, dtype=torch.float64, device=dev)
        self.bR = torch.zeros(C, mR, dtype=torch.float64, device=dev)
        self.binfo = torch.zeros(C, dtype=torch.int32, device=dev)
        # -1/2 (sum log N + r^T N^-1 r) + 1/2 sum_M log phiinv_M (get_lnlikelihood_fullmarg :583-600)
        Nh, rh = np.asarray(Nvec, float), np.asarray(r, float)
        self.lnl_const = float(-0.5 * (np.sum(np.log(Nh)) + np.sum(rh ** 2 / Nh)) + 0.5 * np.sum(np.log(phf)))

    # ----------------------------------------------------------------- kernels
    def factor(self, x, fused=None):
        """Schur complement of every chain's ECORR state in x (C, n_param) + R prefix: one
        fused launch (gs_ecorr_prefix) when the fixed-prior block fits one 16-column tile,
        else gs_ecorr_schur + gs_prefix_sys."""
        lib, h = self.ctx.lib, self.ctx.handle
        if self.fused if fused is None else fused:
            check(lib.gs_ecorr_prefix(h, self.C, self.NF, self.NMX, self.nm, self.ne, self.ldbp, ptr(self.Bp),
                                      ptr(self.Dg), ptr(self.ebk), self.n_bk, ptr(self.ecol), ptr(x), x.shape[1],
                                      ptr(self.Ap), None, ptr(self.model), ptr(self.aux), None, ptr(self.pinfo),
                                      *self.strides), "gs_ecorr_prefix")
            return
        check(lib.gs_ecorr_schur(h, self.C, self.mR, self.ne, self.ldbx, ptr(self.Bx), ptr(self.Dg), ptr(self.ebk),
                                 self.n_bk, ptr(self.ecol), ptr(x), x.shape[1], ptr(self.A), ptr(self.dR),
                                 ptr(self.TNTc), ptr(self.dc), ptr(self.aux)), "gs_ecorr_schur")
        check(lib.gs_prefix_sys(h, 1, self.C, self.NF, self.NMX, ptr(self.pdesc), self.mR * self.mR, self.mR,
                                ptr(self.TNTc), ptr(self.dc), ptr(self.fidx), ptr(self.midx), ptr(self.phfix),
                                ptr(self.model), ptr(self.pinfo)), "gs_prefix_sys")

    def gather(self, TNT, d, tnt_cstride, d_cstride):
        """Per-chain [B | d_E], Dg, Ap from per-chain TNT / d (white.WhiteNoiseModel.tnt)."""
        check(self.ctx.lib.gs_ecorr_gather(self.ctx.handle, self.C, self.m, self.ne, self.ldbp, ptr(self.ecid),
                                           ptr(self.colmap), ptr(self.phm), ptr(TNT), tnt_cstride, ptr(d),
                                           d_cstride, ptr(self.Bp), ptr(self.Dg), ptr(self.Ap)), "gs_ecorr_gather")

    def gather_R(self, TNT_R, d_R, tnt_cstride, d_cstride):
        """Per-chain Ap from the per-chain TNT / d of the R columns only (rc order)."""
        if not hasattr(self, "colmap_R"):
            cm = self.jmap.clone()
            cm[self.dcol] = -2
            self.colmap_R = cm.contiguous()
        check(self.ctx.lib.gs_ecorr_gather(self.ctx.handle, self.C, self.mR, 0, self.ldbp, ptr(self.ecid),
                                           ptr(self.colmap_R), ptr(self.phm), ptr(TNT_R), tnt_cstride, ptr(d_R),
                                           d_cstride, ptr(self.Bp), ptr(self.Dg), ptr(self.Ap)), "gs_ecorr_gather")

    def _eval(self, x, phiinv_F):
        """lnl / aux / info of every chain at x: one fused likelihood-mode launch when
        available (no model block), else factor + gs_lnlike_marg."""
        if self.fused and self.fused_lnl:
            if self._linfo_dirty:   # the likelihood-mode kernel reports through pinfo only
                self.linfo.zero_()
                self._linfo_dirty = False
            check(self.ctx.lib.gs_ecorr_prefix(self.ctx.handle, self.C, self.NF, self.NMX, self.nm, self.ne,
                                               self.ldbp, ptr(self.Bp), ptr(self.Dg), ptr(self.ebk), self.n_bk,
                                               ptr(self.ecol), ptr(x), x.shape[1], ptr(self.Ap), ptr(phiinv_F),
                                               None, ptr(self.aux), ptr(self.lnl), ptr(self.pinfo),
                                               *self.strides), "gs_ecorr_prefix")
            return
        self.factor(x)
        self._lnl_R(phiinv_F)
        self._linfo_dirty = True

    def _lnl_R(self, phiinv_F):
        check(self.ctx.lib.gs_lnlike_marg(self.ctx.handle, 1, self.C, self.NF, self.NMX, ptr(self.model), 1,
                                          ptr(self.nm_dev), ptr(phiinv_F), ptr(self.lnl), ptr(self.linfo)),
              "gs_lnlike_marg")

    def lnlike(self, x, phiinv_F, lnl_const=None):
        """get_lnlikelihood_fullmarg (pulsar_gibbs.py:569-610) of every chain: (C,) tensor.
        lnl_const: -1/2 (sum log N + r^T N^-1 r) + 1/2 sum_M log phiinv_M per chain when N
        differs per chain (default: the model's fixed-N value)."""
        self._eval(x, phiinv_F)
        a = self.aux
        ok = (self.pinfo == 0) & (self.linfo == 0)
        const = self.lnl_const if lnl_const is None else lnl_const
        val = self.lnl + 0.5 * (a[:, 1] - a[:, 0] - a[:, 2]) + const
        return torch.where(ok, val, torch.full_like(val, -np.inf))

    REFRESH = 64   # incremental steps between full evaluations of the state (rounding does not pile up)

    def _state_buffers(self):
        if not hasattr(self, "tbuf"):
            nb = self.ldbp // 16
            nt = nb * (nb + 1) // 2
            self.tbuf = torch.empty(2, self.C, nt * 256, dtype=torch.float64, device=self.ctx.device)
            self.tidx = torch.zeros(self.C, dtype=torch.int32, device=self.ctx.device)

    def _eval_state(self, x, phiinv_F, x_old=None):
        """gs_ecorr_lnl_state: lnl / aux / pinfo at x, fully (x_old None: the state slot tidx gets
        T(x)) or as one Metropolis step from the stored state at x_old (the other slot gets T(x))."""
        bs, ds, aps = self.strides
        check(self.ctx.lib.gs_ecorr_lnl_state(
            self.ctx.handle, self.C, self.NF, self.NMX, self.nm, self.ne, self.ldbp, ptr(self.Bp), ptr(self.Dg),
            ptr(self.ebk), self.n_bk, ptr(self.ecol), ptr(self.eoff), ptr(x), ptr(x_old),
            ptr(self.prop) if x_old is not None else None, x.shape[1], ptr(self.Ap), ptr(phiinv_F), ptr(self.tbuf),
            ptr(self.tidx), ptr(self.aux), ptr(self.lnl), ptr(self.pinfo), bs, ds, aps), "gs_ecorr_lnl_state")

    def mh(self, x, phiinv_F, n_steps, sweep=0, chain_base=0, inj=None, q_rec=None, n_acc=None):
        """n_steps Metropolis steps of update_ecorr_params (pulsar_gibbs.py:456-484) for every
        chain, x (C, n_param) updated in place.  inj (n_steps, C, 4) or None (Philox);
        q_rec (n_steps, C, n_e) proposals or None."""
        lib, h = self.ctx.lib, self.ctx.handle
        ne_p = self.n_bk
        n_steps = int(n_steps)
        inc = self.incremental and self.fused and self.fused_lnl
        if inc:
            self._state_buffers()
            if self._linfo_dirty:   # the likelihood-mode kernels report through pinfo only
                self.linfo.zero_()
                self._linfo_dirty = False
            self.tidx.zero_()
            self._eval_state(x, phiinv_F)
        else:
            self._eval(x, phiinv_F)
        tidx = self.tidx if inc else None

        # each accept launch also draws the next step's proposal (gs_ecorr_accept_propose):
        # init + propose(0), then per step likelihood -> accept(s) + propose(s + 1)
        def accept_propose(init, qr, nxt):
            check(lib.gs_ecorr_accept_propose2(
                h, self.C, ne_p, ptr(self.ecol), init, ptr(self.lnl), ptr(self.linfo), ptr(self.pinfo),
                ptr(self.aux), ptr(self.prop), ptr(self.xq), ptr(x), x.shape[1], ptr(self.lnl0), ptr(qr),
                None if init else ptr(n_acc), ptr(self.emin), ptr(self.emax), self.n_param, nxt, sweep,
                chain_base, ptr(inj), ptr(tidx)), "gs_ecorr_accept_propose2")

        accept_propose(1, None, 0 if n_steps > 0 else -1)
        for s in range(n_steps):
            if inc:
                if s and s % self.REFRESH == 0:
                    self._eval_state(x, phiinv_F)          # re-base the state at x (lnl0 kept)
                self._eval_state(self.xq, phiinv_F, x_old=x)
            else:
                self._eval(self.xq, phiinv_F)
            accept_propose(0, q_rec[s] if q_rec is not None else None, s + 1 if s + 1 < n_steps else -1)

    def bdraw(self, x, phiinv_F, b, z=None, sweep=0, first=False, chain_base=0, chain_mask=None):
        """b | rho, ECORR of every chain (update_b, pulsar_gibbs.py:489-520): b (C, ldb >= m)
        written in original column order (masked chains keep theirs).  z (C, m) injected
        normals by original column, or None (Philox)."""
        lib, h = self.ctx.lib, self.ctx.handle
        self.factor(x)
        zR = z[:, torch.as_tensor(self.rc_host, device=z.device)].contiguous() if z is not None else None
        ev_r = _lib.EV_B0 if first else _lib.EV_B
        ev_e = _lib.EV_ECORR_B0 if first else _lib.EV_ECORR_B
        check(lib.gs_bdraw_sys(h, 1, self.C, self.NF, self.NMX, self.mR, ptr(self.model), ptr(self.fidx),
                               ptr(self.midx), ptr(self.nm_dev), ptr(phiinv_F), ptr(zR), sweep, ev_r, chain_base,
                               ptr(chain_mask), ptr(self.bR), ptr(self.binfo)), "gs_bdraw_sys")
        if self.fused:   # reordered [M | F | d] rows (shared or per chain)
            Bx, ldbx, dcol, jmap = self.Bp, self.ldbp, self.dcol, self.jmap
        else:
            if not hasattr(self, "_jmap_r"):
                self._jmap_r = torch.arange(self.mR, dtype=torch.int32, device=x.device)
                self._jmap_r = torch.cat([self._jmap_r, torch.full((self.ldbx - self.mR,), -1, dtype=torch.int32,
                                                                   device=x.device)])
            Bx, ldbx, dcol, jmap = self.Bx, self.ldbx, self.mR, self._jmap_r
        check(lib.gs_ecorr_bdraw_e(h, self.C, self.mR, self.ne, ldbx, ptr(Bx), ptr(self.Dg), ptr(self.ebk),
                                   ptr(self.ecol), ptr(x), x.shape[1], ptr(self.bR), self.mR, ptr(self.ecid),
                                   ptr(self.rcol), self.m, ptr(z), sweep, ev_e, chain_base, ptr(chain_mask), ptr(b),
                                   b.shape[1], self.strides[0], self.strides[1], dcol, ptr(jmap)),
              "gs_ecorr_bdraw_e")
        return b


class EcorrFreeSpectrumChains:
    """n_chain chains of one pulsar with the basis-ECORR MH block and the analytic free
    spectrum, in the notebook sampler's order (pta_gibbs_freespec.ipynb cell 2 sample();
    pulsar_gibbs.py:656-698 with the ECORR block of :675-683 enabled):

        record x, b -> [ii == 0: b from x0] -> ECORR MH (aclength_ecorr steps) -> rho|b
        -> gate all(xnew != x_old[-1]) -> b|rho
    """

    WARMUP = 1000   # update_ecorr_params(xnew, iters=1000) at ii == 0 (notebook sample())

    def __init__(self, em: EcorrModel, gw_cols, gwid, rhomin, rhomax, x0, aclength=None, chain_base=0):
        self.em = em
        self.ctx = em.ctx
        dev = self.ctx.device
        C = em.C
        self.gw_cols = _t(np.asarray(gw_cols, np.int32), torch.int32, dev)
        self.gw_cols_host = np.asarray(gw_cols, np.int64)
        self.gw0 = int(self.gw_cols_host[0])
        if not np.array_equal(self.gw_cols_host, self.gw0 + np.arange(em.NF // 2)):
            raise NotImplementedError("the gw log10_rho columns must be contiguous in x")
        self.fidx_full = _t(np.asarray(gwid, np.int32)[None, :], torch.int32, dev)
        self.rhomin, self.rhomax = float(rhomin), float(rhomax)
        self.aclength = None if aclength is None else int(aclength)
        self.short_chain = None
        self.chain_base = int(chain_base)
        self.x = _t(np.broadcast_to(np.asarray(x0, float), (C, em.n_param)), torch.float64, dev)
        self.ldb = em.m
        self.b = torch.zeros(C, self.ldb, dtype=torch.float64, device=dev)
        self.phiinv_F = torch.empty(C, em.NF, dtype=torch.float64, device=dev)
        self.xlast = torch.empty(C, dtype=torch.float64, device=dev)
        self.gate = torch.empty(C, dtype=torch.int32, device=dev)
        self.n_acc = torch.zeros(C, dtype=torch.int32, device=dev)
        self.it = 0

    def _phiinv(self, with_gate):
        check(self.ctx.lib.gs_pta_gate_phiinv(self.ctx.handle, 1, self.em.C, self.em.NF // 2, self.em.n_param,
                                              ptr(self.x), ptr(self.xlast) if with_gate else None,
                                              ptr(self.gw_cols), None, ptr(self.phiinv_F), ptr(self.gate)),
              "gs_pta_gate_phiinv")

    def sweep(self, x_rec=None, b_rec=None, z0=None, z=None, u=None, mh_inj=None):
        """One sweep of every chain; x_rec / b_rec (C, n_param) / (C, ldb) get the state
        before the update (pulsar_gibbs.py:658-659)."""
        em, lib, h = self.em, self.ctx.lib, self.ctx.handle
        ii = self.it
        if x_rec is not None:
            x_rec.copy_(self.x)
        if b_rec is not None:
            b_rec.copy_(self.b)
        self.xlast.copy_(self.x[:, -1])
        if ii == 0:  # first b from xs (:661-662)
            self._phiinv(False)
            em.bdraw(self.x, self.phiinv_F, self.b, z=z0, sweep=ii, first=True, chain_base=self.chain_base)
        self._phiinv(False)
        if self.aclength is None:
            # warm-up (update_ecorr_params iters=1000, pulsar_gibbs.py:422-451): the proposals
            # q[eind] form short_chain; aclength_ecorr = max acor over its columns after 100
            # (chain 0's value is used by every chain)
            from .diagnostics import white_aclength
            q_rec = torch.empty(self.WARMUP, em.C, em.n_bk, dtype=torch.float64, device=self.ctx.device)
            em.mh(self.x, self.phiinv_F, self.WARMUP, sweep=ii, chain_base=self.chain_base, q_rec=q_rec,
                  n_acc=self.n_acc)
            self.short_chain = q_rec[:, 0].cpu().numpy()
            self.aclength = int(white_aclength(self.short_chain))
        else:
            em.mh(self.x, self.phiinv_F, self.aclength, sweep=ii, chain_base=self.chain_base, inj=mh_inj,
                  n_acc=self.n_acc)
        # rho|b writes the n_f log10_rho columns of x in place (:206-216, 236)
        xg = ctypes.c_void_p(self.x.data_ptr() + 8 * self.gw0)
        check(lib.gs_rho_analytic(h, 1, em.C, em.NF, self.ldb, ptr(self.fidx_full), ptr(self.b), ptr(u), ii,
                                  self.chain_base, self.rhomin, self.rhomax, xg, em.n_param), "gs_rho_analytic")
        self._phiinv(True)
        em.bdraw(self.x, self.phiinv_F, self.b, z=z, sweep=ii, chain_base=self.chain_base, chain_mask=self.gate)
        self.it += 1


class EcorrWhiteChains:
    """White noise AND basis ECORR sampled (the notebook's J1713 run, white_vary=True), n_chain
    chains of one pulsar, in the notebook sampler's order (pta_gibbs_freespec.ipynb cell 2):

        record x, b -> [ii == 0: b from x0] -> white MH on y = r - T b (pulsar_gibbs.py:373-404)
        -> TNT_c, d_c with the chain's new N (gs_white_tnt: the reference's TNT reset + the
        recompute inside get_lnlikelihood) -> per-chain ECORR operands (gs_ecorr_gather)
        -> ECORR MH (:456-484) -> rho|b -> gate -> b|rho

    wm: white.WhiteNoiseModel(prefix=False) over the full basis; em: EcorrModel(per_chain=True).
    """

    def __init__(self, wm, em: EcorrModel, gw_cols, gwid, rhomin, rhomax, x0, aclength_white,
                 aclength_ecorr, chain_base=0, wmR=None):
        if not em.per_chain:
            raise ValueError("EcorrWhiteChains needs EcorrModel(per_chain=True)")
        self.wm, self.em, self.ctx = wm, em, em.ctx
        # wmR (white.WhiteNoiseModel over the R columns only): TNT_RR by the batched SYRK and
        # the epoch rows by segment sums (gs_ecorr_epoch_sums) instead of the full m x m SYRK
        self.wmR = wmR
        if wmR is not None:
            self._epoch_lists()
        dev = self.ctx.device
        C = em.C
        gw = np.asarray(gw_cols, np.int64)
        self.gw0 = int(gw[0])
        if not np.array_equal(gw, self.gw0 + np.arange(em.NF // 2)):
            raise NotImplementedError("the gw log10_rho columns must be contiguous in x")
        self.gw_cols = _t(gw.astype(np.int32), torch.int32, dev)
        self.fidx_full = _t(np.asarray(gwid, np.int32)[None, :], torch.int32, dev)
        self.rhomin, self.rhomax = float(rhomin), float(rhomax)
        self.acl_w, self.acl_e = int(aclength_white), int(aclength_ecorr)
        self.chain_base = int(chain_base)
        self.x = _t(np.broadcast_to(np.asarray(x0, float), (C, em.n_param)), torch.float64, dev)
        self.b = torch.zeros(C, em.m, dtype=torch.float64, device=dev)
        self.phiinv_F = torch.empty(C, em.NF, dtype=torch.float64, device=dev)
        self.xlast = torch.empty(C, dtype=torch.float64, device=dev)
        self.gate = torch.empty(C, dtype=torch.int32, device=dev)
        self.n_acc_white = torch.zeros(C, dtype=torch.int32, device=dev)
        self.n_acc_ecorr = torch.zeros(C, dtype=torch.int32, device=dev)
        self.it = 0

    def _phiinv(self, with_gate):
        em = self.em
        check(self.ctx.lib.gs_pta_gate_phiinv(self.ctx.handle, 1, em.C, em.NF // 2, em.n_param, ptr(self.x),
                                              ptr(self.xlast) if with_gate else None, ptr(self.gw_cols), None,
                                              ptr(self.phiinv_F), ptr(self.gate)), "gs_pta_gate_phiinv")

    def _epoch_lists(self):
        """CSR lists (TOA, u) of every epoch column in wm's (backend-grouped) TOA order."""
        wm, em, dev = self.wm, self.em, self.ctx.device
        n, m = int(wm.n_toa[0]), em.m
        Tp = wm.T[:n * m].view(n, m)
        U = Tp[:, torch.as_tensor(em.ecid_host, device=dev)].cpu().numpy()
        ptr_, toa, val = [0], [], []
        for e in range(em.ne):
            nz = np.nonzero(U[:, e])[0]
            toa += list(nz)
            val += list(U[nz, e])
            ptr_.append(len(toa))
        self.eptr = _t(np.asarray(ptr_, np.int32), torch.int32, dev)
        self.etoa = _t(np.asarray(toa, np.int32), torch.int32, dev)
        self.eu = _t(np.asarray(val, float), torch.float64, dev)

    def _operands(self):
        wm, em = self.wm, self.em
        if self.wmR is None:
            wm.tnt(self.x, em.n_param)
            em.gather(wm.TNT, wm.d, wm.tnt_cstride, wm.d_cstride)
            return
        wmR = self.wmR
        wmR.tnt(self.x, em.n_param)
        em.gather_R(wmR.TNT, wmR.d, wmR.tnt_cstride, wmR.d_cstride)
        check(self.ctx.lib.gs_ecorr_epoch_sums(
            self.ctx.handle, em.C, ptr(wm.wdesc), ptr(wm.wcol), ptr(wm.wkind), ptr(wm.wbk), ptr(self.x), em.n_param,
            ptr(wm.T), em.m, ptr(wm.sigma2), ptr(wm.bk), ptr(wm.r), em.ne, em.ldbp, em.dcol, ptr(em.colmap),
            ptr(self.eptr), ptr(self.etoa), ptr(self.eu), ptr(em.Bp), ptr(em.Dg)), "gs_ecorr_epoch_sums")

    def sweep(self, x_rec=None, b_rec=None, z0=None, z=None, u=None, white_inj=None, ecorr_inj=None):
        em, wm, lib, h = self.em, self.wm, self.ctx.lib, self.ctx.handle
        ii = self.it
        if x_rec is not None:
            x_rec.copy_(self.x)
        if b_rec is not None:
            b_rec.copy_(self.b)
        self.xlast.copy_(self.x[:, -1])
        if ii == 0:
            self._operands()
            self._phiinv(False)
            em.bdraw(self.x, self.phiinv_F, self.b, z=z0, sweep=ii, first=True, chain_base=self.chain_base)
        wm.resid(self.b)
        wm.mh(self.x, em.n_param, self.acl_w, ii, chain_base=self.chain_base, inj=white_inj, n_acc=self.n_acc_white)
        self._operands()
        self._phiinv(False)
        em.mh(self.x, self.phiinv_F, self.acl_e, sweep=ii, chain_base=self.chain_base, inj=ecorr_inj,
              n_acc=self.n_acc_ecorr)
        xg = ctypes.c_void_p(self.x.data_ptr() + 8 * self.gw0)
        check(lib.gs_rho_analytic(h, 1, em.C, em.NF, em.m, ptr(self.fidx_full), ptr(self.b), ptr(u), ii,
                                  self.chain_base, self.rhomin, self.rhomax, xg, em.n_param), "gs_rho_analytic")
        self._phiinv(True)
        em.bdraw(self.x, self.phiinv_F, self.b, z=z, sweep=ii, chain_base=self.chain_base, chain_mask=self.gate)
        self.it += 1


def white_ecorr_models(ctx, T, r, sigma, backends, gwid, white_list, ecid, epoch_backend, ecol, emin, emax,
                       n_param, n_chain, phiinv_fixed=1e-40):
    """(wm, wmR, em) for EcorrWhiteChains: the white model over the full basis (residuals,
    white MH), the white model over the R columns (TNT_RR), the per-chain ECORR model."""
    from .white import WhiteNoiseModel
    T = np.ascontiguousarray(T, float)
    m = T.shape[1]
    gwid = np.asarray(gwid)
    rc = np.setdiff1d(np.arange(m), np.asarray(ecid))
    pos = {c: i for i, c in enumerate(rc)}
    nfix = m - gwid.size
    wm = WhiteNoiseModel(ctx, [T], [r], [sigma], [backends], [gwid], [np.full(nfix, 1e-40)], [white_list],
                         n_chain, prefix=False)
    wmR = WhiteNoiseModel(ctx, [np.ascontiguousarray(T[:, rc])], [r], [sigma], [backends],
                          [np.array([pos[c] for c in gwid])], [np.full(rc.size - gwid.size, 1e-40)], [white_list],
                          n_chain, prefix=False)
    em = EcorrModel(ctx, T, np.asarray(sigma, float) ** 2, r, ecid, epoch_backend, gwid, ecol, emin, emax, n_param,
                    n_chain, phiinv_fixed=phiinv_fixed, per_chain=True)
    return wm, wmR, em
