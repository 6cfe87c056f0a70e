"""Device state of white-noise Gibbs runs (row a10; configs 5 and single pulsars with
varied EFAC/EQUAD).

When white-noise parameters are sampled, N — and with it TNT, d and the Cholesky
prefix — differs per chain and changes every sweep (pulsar_gibbs.py:495-502, reset
:664-665).  ``WhiteNoiseModel`` keeps, per pulsar, T (row-major for the TNT MFMA
kernel and column-major for y = r - T b), r, sigma^2 and the backend of every TOA
with the TOAs grouped by backend, plus per-(pulsar, chain) TNT / d / model blocks.

``WhiteFreeSpectrumChains`` runs PulsarBlockGibbs.sample's loop body
(pulsar_gibbs.py:656-698) for n_chain chains of one pulsar with a white-noise MH
block and the analytic free-spectrum rho draw:

    record x, b -> [ii == 0: b from x0] -> y = r - T b -> white MH (1000 warm-up
    steps at ii == 0, then aclength_white steps) -> rho|b -> gate -> TNT_c, prefix_c
    -> gated b|rho.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _lib
from ._lib import check, ptr
from .diagnostics import white_aclength
from .engine import BIG_NF, _t, nf_supported

MAX_BK = 15
MAX_W = 32
KIND = {"efac": 0, "tnequad": 1, "t2equad": 2}

WHITE_DESC = np.dtype([("n_toa", np.int64), ("toa_off", np.int64), ("w_off", np.int64),
                       ("n_bk", np.int32), ("n_w", np.int32), ("bk_off", np.int32, (MAX_BK + 1,))])
assert WHITE_DESC.itemsize == 96


def white_kind(name):
    """GS_WHITE_* kind of a white-noise parameter name (efac, log10_tnequad, log10_t2equad;
    enterprise's plain 'equad' adds in quadrature like tnequad)."""
    if name.endswith("efac"):
        return KIND["efac"]
    if "t2equad" in name:
        return KIND["t2equad"]
    if "equad" in name:
        return KIND["tnequad"]
    raise ValueError(f"not a white-noise parameter: {name}")


class WhiteNoiseModel:
    """Per-pulsar TOA data + per-(pulsar, chain) TNT / d / prefix model blocks.

    T_list[p] (n_toa x m), r_list[p], sigma_list[p] (TOA errors), backend_list[p]
    (int per TOA), fidx_list[p] (NF gwid columns), phiinv_fixed_list[p] (phiinv of the
    other columns in increasing order), white_list[p]: [(x column, kind, backend,
    pmin, pmax)] for the pulsar's white parameters in x order (wind order).
    """

    def __init__(self, ctx, T_list, r_list, sigma_list, backend_list, fidx_list, phiinv_fixed_list,
                 white_list, n_chain, prefix=True):
        self.ctx = ctx
        dev = ctx.device
        P = len(T_list)
        C = int(n_chain)
        NF = len(fidx_list[0])
        if any(len(f) != NF for f in fidx_list):
            raise ValueError("every pulsar must have the same number of free-spectrum columns")
        if not nf_supported(NF):
            raise NotImplementedError(f"NF = 2*n_f = {NF}; supported: even NF <= {BIG_NF[1]}")
        self.P, self.C, self.NF = P, C, NF
        self.m = np.array([t.shape[1] for t in T_list], np.int64)
        self.n_toa = np.array([t.shape[0] for t in T_list], np.int64)
        self.nm = (self.m - NF).astype(np.int32)
        # prefix=False: per-chain TNT / d, residuals and the white MH only (the basis-ECORR
        # path factors its own Schur systems, ecorr.EcorrModel(per_chain=True))
        self.prefix = bool(prefix)
        if self.prefix and ((self.nm < 0).any() or (self.nm > 64).any()):
            raise NotImplementedError("need 0..64 fixed-prior columns per pulsar")
        self.NMX = int(self.nm.max())
        self.ldb = max(int(self.m.max()), NF + 1)    # the C-ABI wants ldb > NF (nm = 0 models)
        fidx = np.zeros((P, NF), np.int32)
        midx = np.zeros((P, max(1, self.NMX)), np.int32)      # one unused column when nm = 0
        phfix = np.ones((P, max(1, self.NMX)))
        self.perm = []
        Ts, Tts, rs, s2s, bks = [], [], [], [], []
        wdesc = np.zeros(P, WHITE_DESC)
        wcol, wkind, wbk, wmin, wmax = [], [], [], [], []
        toa_off = np.concatenate([[0], np.cumsum(self.n_toa)])[:-1]
        for p in range(P):
            mask = np.ones(self.m[p], bool)
            mask[np.asarray(fidx_list[p])] = False
            mi = np.nonzero(mask)[0]
            fidx[p] = fidx_list[p]
            midx[p, :mi.size] = mi
            phfix[p, :mi.size] = phiinv_fixed_list[p]
            bk = np.asarray(backend_list[p], np.int64)
            nbk = int(bk.max()) + 1
            if nbk > MAX_BK:
                raise NotImplementedError(f"more than {MAX_BK} backends")
            perm = np.argsort(bk, kind="stable")       # group TOAs by backend
            self.perm.append(perm)
            T = np.asarray(T_list[p], float)[perm]
            Ts.append(T.ravel())
            Tts.append(np.ascontiguousarray(T.T).ravel())
            rs.append(np.asarray(r_list[p], float)[perm])
            s2s.append(np.asarray(sigma_list[p], float)[perm] ** 2)
            bks.append(bk[perm].astype(np.int32))
            counts = np.bincount(bk, minlength=nbk)
            wl = list(white_list[p])
            if len(wl) > MAX_W:
                raise NotImplementedError(f"more than {MAX_W} white parameters per pulsar")
            d = wdesc[p]
            d["n_toa"], d["toa_off"], d["w_off"] = self.n_toa[p], toa_off[p], len(wcol)
            d["n_bk"], d["n_w"] = nbk, len(wl)
            d["bk_off"][:nbk + 1] = np.concatenate([[0], np.cumsum(counts)])
            for col, kind, k, lo, hi in wl:
                wcol.append(col)
                wkind.append(kind)
                wbk.append(k)
                wmin.append(lo)
                wmax.append(hi)
        self.n_w = np.array([len(w) for w in white_list])
        T_off = np.concatenate([[0], np.cumsum(self.n_toa * self.m)])[:-1]
        tnt_off = np.concatenate([[0], np.cumsum(self.m * self.m)])[:-1]
        d_off = np.concatenate([[0], np.cumsum(self.m)])[:-1]
        self.tnt_cstride = int(np.sum(self.m * self.m))
        self.d_cstride = int(np.sum(self.m))
        self.tnt_off, self.d_off = tnt_off, d_off
        tdesc = np.stack([self.n_toa, self.m, T_off, toa_off, tnt_off, d_off], axis=1).astype(np.int64)
        pdesc = np.stack([self.m, self.nm.astype(np.int64), tnt_off, d_off], axis=1).astype(np.int64)
        self.ntot = int(self.n_toa.sum())
        self.T = _t(np.concatenate(Ts), torch.float64, dev)
        self.Tt = _t(np.concatenate(Tts), torch.float64, dev)
        self.r = _t(np.concatenate(rs), torch.float64, dev)
        self.sigma2 = _t(np.concatenate(s2s), torch.float64, dev)
        self.bk = _t(np.concatenate(bks), torch.int32, dev)
        self.tdesc = _t(tdesc, torch.int64, dev)
        self.pdesc = _t(pdesc, torch.int64, dev)
        self.wdesc = _t(wdesc.view(np.int64).reshape(P, -1), torch.int64, dev)
        self.wcol = _t(np.asarray(wcol, np.int32), torch.int32, dev)
        self.wkind = _t(np.asarray(wkind, np.int32), torch.int32, dev)
        self.wbk = _t(np.asarray(wbk, np.int32), torch.int32, dev)
        self.wmin = _t(np.asarray(wmin, float), torch.float64, dev)
        self.wmax = _t(np.asarray(wmax, float), torch.float64, dev)
        self.fidx = _t(fidx, torch.int32, dev)
        self.midx = _t(midx, torch.int32, dev)
        self.nm_dev = _t(self.nm, torch.int32, dev)
        self.phfix = _t(phfix, torch.float64, dev)
        self.mstride = int(ctx.lib.gs_model_stride(NF, self.NMX))
        self.TNT = torch.empty(C * self.tnt_cstride, dtype=torch.float64, device=dev)
        self.d = torch.empty(C * self.d_cstride, dtype=torch.float64, device=dev)
        self.model = torch.empty(P * C * self.mstride if self.prefix else 0, dtype=torch.float64, device=dev)
        self.y = torch.empty(C, self.ntot, dtype=torch.float64, device=dev)
        self.pinfo = torch.zeros(P * C, dtype=torch.int32, device=dev)

    # ---------------------------------------------------------------- kernels
    def tnt(self, x, ldx):
        """TNT_c, d_c from the white parameters in x (pulsar_gibbs.py:495-502)."""
        check(self.ctx.lib.gs_white_tnt(self.ctx.handle, self.P, self.C, int(self.m.max()), ptr(self.tdesc),
                                        ptr(self.wdesc), ptr(self.wcol), ptr(self.wkind), ptr(self.wbk),
                                        ptr(self.T), ptr(self.sigma2), ptr(self.bk), ptr(self.r), ptr(x), ldx,
                                        self.tnt_cstride, self.d_cstride, ptr(self.TNT), ptr(self.d)),
              "gs_white_tnt")

    def refresh(self, x, ldx):
        """TNT_c, d_c from the white parameters in x, then the per-system prefix."""
        lib, h = self.ctx.lib, self.ctx.handle
        check(lib.gs_white_tnt(h, self.P, self.C, int(self.m.max()), ptr(self.tdesc), ptr(self.wdesc),
                               ptr(self.wcol), ptr(self.wkind), ptr(self.wbk), ptr(self.T), ptr(self.sigma2),
                               ptr(self.bk), ptr(self.r), ptr(x), ldx, self.tnt_cstride, self.d_cstride,
                               ptr(self.TNT), ptr(self.d)), "gs_white_tnt")
        check(lib.gs_prefix_sys(h, self.P, self.C, self.NF, self.NMX, ptr(self.pdesc), self.tnt_cstride,
                                self.d_cstride, ptr(self.TNT), ptr(self.d), ptr(self.fidx), ptr(self.midx),
                                ptr(self.phfix), ptr(self.model), ptr(self.pinfo)), "gs_prefix_sys")

    def resid(self, b):
        check(self.ctx.lib.gs_white_resid(self.ctx.handle, self.P, self.C, int(self.n_toa.max()), self.ldb,
                                          ptr(self.tdesc), ptr(self.Tt), ptr(self.r), ptr(b), self.ntot,
                                          ptr(self.y)), "gs_white_resid")

    def mh(self, x, ldx, n_steps, sweep, chain_base=0, nsteps_chain=None, inj=None, q_rec=None, n_acc=None):
        check(self.ctx.lib.gs_white_mh(self.ctx.handle, self.P, self.C, ptr(self.wdesc), ptr(self.wcol),
                                       ptr(self.wkind), ptr(self.wbk), ptr(self.wmin), ptr(self.wmax),
                                       ptr(self.sigma2), ptr(self.y), self.ntot, ptr(x), ldx, int(n_steps),
                                       ptr(nsteps_chain), sweep, chain_base, ptr(inj), ptr(q_rec),
                                       ptr(n_acc)), "gs_white_mh")

    def bdraw(self, phiinv_F, b, info, z=None, sweep=0, event=_lib.EV_B, chain_base=0, chain_mask=None):
        check(self.ctx.lib.gs_bdraw_sys(self.ctx.handle, self.P, self.C, self.NF, self.NMX, self.ldb,
                                        ptr(self.model), ptr(self.fidx), ptr(self.midx), ptr(self.nm_dev),
                                        ptr(phiinv_F), ptr(z), sweep, event, chain_base, ptr(chain_mask),
                                        ptr(b), ptr(info)), "gs_bdraw_sys")

    def tnt_host(self, p, c):
        m = int(self.m[p])
        o = int(self.tnt_off[p]) + c * self.tnt_cstride
        od = int(self.d_off[p]) + c * self.d_cstride
        return self.TNT[o:o + m * m].view(m, m).cpu().numpy(), self.d[od:od + m].cpu().numpy()


class WhiteFreeSpectrumChains:
    """n_chain chains of one pulsar with white-noise MH + analytic free spectrum.

    x (n_chain, n_param) in the PTA's parameter order, b (n_chain, ldb) in the
    pulsar's ORIGINAL column order.  gw_cols: the n_f log10_rho columns of x.
    """

    WARMUP = 1000   # update_white_params(xnew, iters=1000) at ii == 0 (pulsar_gibbs.py:669-670)

    def __init__(self, wm: WhiteNoiseModel, n_param, gw_cols, rhomin, rhomax, x0, chain_base=0,
                 aclength=None):
        if wm.P != 1:
            raise ValueError("WhiteFreeSpectrumChains drives one pulsar")
        self.wm, self.ctx = wm, wm.ctx
        dev = self.ctx.device
        C = wm.C
        self.C, self.n_param = C, int(n_param)
        self.n_f = wm.NF // 2
        gw_cols = np.asarray(gw_cols, np.int64)
        if not np.array_equal(gw_cols, gw_cols[0] + np.arange(self.n_f)):
            raise NotImplementedError("log10_rho columns must be contiguous in x")
        self.gw0 = int(gw_cols[0])
        self.gw_col = _t(gw_cols.astype(np.int32), torch.int32, dev)
        self.rhomin, self.rhomax = float(rhomin), float(rhomax)
        self.chain_base = int(chain_base)
        self.x = _t(np.broadcast_to(np.asarray(x0, float), (C, self.n_param)), torch.float64, dev)
        self.b = torch.zeros(C, wm.ldb, dtype=torch.float64, device=dev)
        self.phiinv_F = torch.empty(C, wm.NF, dtype=torch.float64, device=dev)
        self.gate = torch.ones(C, dtype=torch.int32, device=dev)
        self.xlast = torch.empty(C, dtype=torch.float64, device=dev)
        self.info = torch.zeros(C, dtype=torch.int32, device=dev)
        self.n_acc = torch.zeros(C, dtype=torch.int32, device=dev)
        self.aclength = aclength          # int, or per-chain array after the warm-up
        self.nsteps_dev = None
        self.short_chain = None
        self.it = 0

    def _gate_phiinv(self, with_gate):
        check(self.ctx.lib.gs_pta_gate_phiinv(
            self.ctx.handle, 1, self.C, self.n_f, self.n_param, ptr(self.x),
            ptr(self.xlast) if with_gate else None, ptr(self.gw_col), None,
            ptr(self.phiinv_F), ptr(self.gate)), "gs_pta_gate_phiinv")

    def set_aclength(self, acl):
        acl = np.atleast_1d(np.asarray(acl, np.int64))
        if acl.size == 1:
            self.aclength = int(acl[0])
            self.nsteps_dev = None
        else:
            self.aclength = acl
            self.nsteps_dev = _t(acl.astype(np.int32), torch.int32, self.ctx.device)

    def sweep(self, x_rec=None, b_rec=None, z0=None, z=None, u=None, mh_inj=None, warmup=None):
        """One sweep for every chain.  Injected draws (parity mode): z0/z (C, ldb) normals
        in original column order, u (C, n_f) uniforms, mh_inj (steps, C, 4)."""
        wm, lib, h = self.wm, self.ctx.lib, self.ctx.handle
        ii = self.it
        check(lib.gs_pta_record(h, self.C, self.n_param, ptr(self.x), ptr(x_rec), ptr(self.xlast)),
              "gs_pta_record")                                     # pulsar_gibbs.py:658
        if b_rec is not None:
            b_rec.copy_(self.b)                                    # :659
        if ii == 0:                                                # :661-662
            wm.refresh(self.x, self.n_param)
            self._gate_phiinv(with_gate=False)
            wm.bdraw(self.phiinv_F, self.b, self.info, z=z0, sweep=ii, event=_lib.EV_B0,
                     chain_base=self.chain_base)
        wm.resid(self.b)                                           # y = r - T b (:534-535)
        if ii == 0 and self.aclength is None:                      # warm-up, :355-371
            n = self.WARMUP if warmup is None else int(warmup)
            q_rec = torch.empty(n, self.C, MAX_W, dtype=torch.float64, device=self.ctx.device)
            wm.mh(self.x, self.n_param, n, ii, self.chain_base, inj=mh_inj, q_rec=q_rec, n_acc=self.n_acc)
            nw = int(wm.n_w[0])
            sc = q_rec[:, :, :nw].cpu().numpy()
            self.short_chain = sc[:, 0, :]
            self.set_aclength([white_aclength(sc[:, c, :]) for c in range(self.C)])
        else:                                                      # :373-404
            steps = int(np.max(self.aclength))
            wm.mh(self.x, self.n_param, steps, ii, self.chain_base, nsteps_chain=self.nsteps_dev,
                  inj=mh_inj, n_acc=self.n_acc)
        check(lib.gs_rho_analytic(h, 1, self.C, wm.NF, wm.ldb, ptr(wm.fidx), ptr(self.b), ptr(u), ii,
                                  self.chain_base, self.rhomin, self.rhomax,
                                  ctypes.c_void_p(self.x.data_ptr() + 8 * self.gw0), self.n_param),
              "gs_rho_analytic")                                   # :206-216, 236
        self._gate_phiinv(with_gate=True)                          # :697
        wm.refresh(self.x, self.n_param)                           # N from the new white params
        wm.bdraw(self.phiinv_F, self.b, self.info, z=z, sweep=ii, event=_lib.EV_B,
                 chain_base=self.chain_base, chain_mask=self.gate)  # :698
        self.it += 1



class WhiteArrayChains:
    """n_chain chains of each of P independent pulsars, each pulsar its own
    PulsarBlockGibbs (white-noise MH + analytic free spectrum): config 5.

    The (pulsar, chain) systems are independent, so x is laid out one row per system,
    x (P * n_chain, n_param) with row p * n_chain + c (GS_OPT_X_PER_SYS on the
    context, which this engine then owns), b (P * n_chain, ldb) in original column
    order.  Every pulsar has the same parameter layout: gw_cols the n_f log10_rho
    columns (contiguous), the white columns given to the WhiteNoiseModel.

    Per sweep, all systems at once (pulsar_gibbs.py:656-698 steady state):
    record -> [ii == 0: TNT, prefix, b from x0] -> y = r - T b -> aclength white MH
    steps -> rho|b -> gate -> TNT_c, d_c (batched SYRK) + prefix -> gated b|rho.
    The reference's 1000-step warm-up (acor) is replaced by a given aclength.
    """

    def __init__(self, wm: WhiteNoiseModel, n_param, gw_cols, rhomin, rhomax, x0, aclength, chain_base=0):
        self.wm, self.ctx = wm, wm.ctx
        dev = self.ctx.device
        self.ctx.set_option(_lib.OPT_X_PER_SYS, 1)
        self.P, self.C = wm.P, wm.C
        self.n_sys = wm.P * wm.C
        self.n_param = int(n_param)
        self.n_f = wm.NF // 2
        gw_cols = np.asarray(gw_cols, np.int64)
        if not np.array_equal(gw_cols, gw_cols[0] + np.arange(self.n_f)):
            raise NotImplementedError("log10_rho columns must be contiguous in x")
        self.gw0 = int(gw_cols[0])
        self.gw_col = _t(gw_cols.astype(np.int32), torch.int32, dev)
        self.rhomin, self.rhomax = float(rhomin), float(rhomax)
        self.chain_base = int(chain_base)
        self.aclength = int(aclength)
        self.x = _t(np.broadcast_to(np.asarray(x0, float), (self.n_sys, self.n_param)), torch.float64, dev)
        self.b = torch.zeros(self.n_sys, wm.ldb, dtype=torch.float64, device=dev)
        self.phiinv_F = torch.empty(self.n_sys, wm.NF, dtype=torch.float64, device=dev)
        self.gate = torch.ones(self.n_sys, dtype=torch.int32, device=dev)
        self.xlast = torch.empty(self.n_sys, dtype=torch.float64, device=dev)
        self.info = torch.zeros(self.n_sys, dtype=torch.int32, device=dev)
        self.n_acc = torch.zeros(self.n_sys, dtype=torch.int32, device=dev)
        self.it = 0

    def _gate_phiinv(self, with_gate):
        check(self.ctx.lib.gs_pta_gate_phiinv(
            self.ctx.handle, 1, self.n_sys, self.n_f, self.n_param, ptr(self.x),
            ptr(self.xlast) if with_gate else None, ptr(self.gw_col), None,
            ptr(self.phiinv_F), ptr(self.gate)), "gs_pta_gate_phiinv")

    def sweep(self, x_rec=None, b_rec=None, z0=None, z=None, u=None, mh_inj=None):
        """One sweep of every system.  Injected draws (parity mode): z0/z (n_sys, ldb),
        u (n_sys, n_f), mh_inj (aclength, n_sys, 4)."""
        wm, lib, h = self.wm, self.ctx.lib, self.ctx.handle
        ii = self.it
        check(lib.gs_pta_record(h, self.n_sys, self.n_param, ptr(self.x), ptr(x_rec), ptr(self.xlast)),
              "gs_pta_record")                                     # pulsar_gibbs.py:658
        if b_rec is not None:
            b_rec.copy_(self.b)                                    # :659
        if ii == 0:                                                # :661-662
            wm.refresh(self.x, self.n_param)
            self._gate_phiinv(with_gate=False)
            wm.bdraw(self.phiinv_F, self.b, self.info, z=z0, sweep=ii, event=_lib.EV_B0,
                     chain_base=self.chain_base)
        wm.resid(self.b)                                           # :534-535
        wm.mh(self.x, self.n_param, self.aclength, ii, self.chain_base, inj=mh_inj,
              n_acc=self.n_acc)                                    # :373-404
        check(lib.gs_rho_analytic(h, self.P, self.C, wm.NF, wm.ldb, ptr(wm.fidx), ptr(self.b), ptr(u), ii,
                                  self.chain_base, self.rhomin, self.rhomax,
                                  ctypes.c_void_p(self.x.data_ptr() + 8 * self.gw0), self.n_param),
              "gs_rho_analytic")                                   # :206-216, 236
        self._gate_phiinv(with_gate=True)                          # :697
        wm.refresh(self.x, self.n_param)
        wm.bdraw(self.phiinv_F, self.b, self.info, z=z, sweep=ii, event=_lib.EV_B,
                 chain_base=self.chain_base, chain_mask=self.gate)  # :698
        self.it += 1
