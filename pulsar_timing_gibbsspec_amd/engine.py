"""Device-resident state for the Gibbs hot path (HBM layout).

* ``DeviceModel`` — per-pulsar TNT/d (gs_tnt) and the fixed-prior Cholesky
  prefix (gs_prefix), built once from the PTA's T, N, r (the reference
  recomputes TNT/d every sweep, pulsar_gibbs.py:664-665; N is fixed in
  configs 1-4 so the result is identical).
* ``FreeSpectrumChains`` — n_chain independent chains per pulsar running the
  fused sweep kernel (gs_sweep_freespec): configs 1-3.
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib
from ._lib import check, ptr

SUPPORTED_NF = (20, 40, 60)


def _t(a, dtype, device):
    return torch.as_tensor(np.ascontiguousarray(a), dtype=dtype).to(device)


class DeviceModel:
    """TNT, d and prefix factors of a ragged batch of pulsars, resident on one GPU.

    T_list[p] (n_toa_p x m_p), N_list[p], r_list[p]: host arrays;
    fidx_list[p]: the NF free-spectrum (gwid) columns in (sin, cos) frequency order;
    phiinv_fixed_list[p]: phiinv of the remaining columns, in increasing column order.
    """

    def __init__(self, ctx, T_list, N_list, r_list, fidx_list, phiinv_fixed_list):
        self.ctx = ctx
        dev = ctx.device
        P = len(T_list)
        NF = len(fidx_list[0])
        if any(len(f) != NF for f in fidx_list):
            raise ValueError("every pulsar must have the same number of free-spectrum columns")
        if NF not in SUPPORTED_NF:
            raise NotImplementedError(f"NF = 2*n_f = {NF}; supported: {SUPPORTED_NF}")
        self.P, self.NF = P, NF
        self.m = np.array([t.shape[1] for t in T_list], np.int64)
        self.n_toa = np.array([t.shape[0] for t in T_list], np.int64)
        self.nm = (self.m - NF).astype(np.int32)
        if (self.nm <= 0).any() or (self.nm > 64).any():
            raise NotImplementedError("need 1..64 fixed-prior columns per pulsar")
        self.NMX = int(self.nm.max())
        self.ldb = int(self.m.max())
        self.fidx_host = [np.asarray(f, np.int64) for f in fidx_list]
        self.midx_host = []
        fidx = np.zeros((P, NF), np.int32)
        midx = np.zeros((P, self.NMX), np.int32)
        phfix = np.ones((P, self.NMX))
        for p in range(P):
            mask = np.ones(self.m[p], bool)
            mask[self.fidx_host[p]] = False
            mi = np.nonzero(mask)[0]
            self.midx_host.append(mi)
            fidx[p] = self.fidx_host[p]
            midx[p, :mi.size] = mi
            phfix[p, :mi.size] = phiinv_fixed_list[p]
        # flat ragged buffers
        T_off = np.concatenate([[0], np.cumsum(self.n_toa * self.m)])[:-1]
        toa_off = np.concatenate([[0], np.cumsum(self.n_toa)])[:-1]
        tnt_off = np.concatenate([[0], np.cumsum(self.m * self.m)])[:-1]
        d_off = np.concatenate([[0], np.cumsum(self.m)])[:-1]
        self.tnt_off, self.d_off = tnt_off, d_off
        tdesc = np.stack([self.n_toa, self.m, T_off, toa_off, tnt_off, d_off], axis=1).astype(np.int64)
        pdesc = np.stack([self.m, self.nm.astype(np.int64), tnt_off, d_off], axis=1).astype(np.int64)
        self.T = _t(np.concatenate([np.ravel(t) for t in T_list]), torch.float64, dev)
        self.Nvec = _t(np.concatenate(N_list), torch.float64, dev)
        self.r = _t(np.concatenate(r_list), torch.float64, dev)
        self.tnt_desc = _t(tdesc, torch.int64, dev)
        self.prefix_desc = _t(pdesc, torch.int64, dev)
        self.TNT = torch.empty(int(np.sum(self.m * self.m)), dtype=torch.float64, device=dev)
        self.d = torch.empty(int(np.sum(self.m)), dtype=torch.float64, device=dev)
        self.fidx = _t(fidx, torch.int32, dev)
        self.midx = _t(midx, torch.int32, dev)
        self.nm_dev = _t(self.nm, torch.int32, dev)
        self.phfix = _t(phfix, torch.float64, dev)
        self.mstride = int(ctx.lib.gs_model_stride(NF, self.NMX))
        self.model = torch.empty(P * self.mstride, dtype=torch.float64, device=dev)
        self.info = torch.zeros(P, dtype=torch.int32, device=dev)
        self.refresh()

    def refresh(self, Nvec=None):
        """(Re)compute TNT/d and the prefix on device (e.g. after a white-noise change)."""
        if Nvec is not None:
            self.Nvec.copy_(_t(np.concatenate(Nvec), torch.float64, self.ctx.device))
        lib, h = self.ctx.lib, self.ctx.handle
        check(lib.gs_tnt(h, self.P, int(self.m.max()), ptr(self.tnt_desc), ptr(self.T), ptr(self.Nvec),
                         ptr(self.r), ptr(self.TNT), ptr(self.d)), "gs_tnt")
        check(lib.gs_prefix(h, self.P, self.NF, self.NMX, ptr(self.prefix_desc), ptr(self.TNT),
                            ptr(self.d), ptr(self.fidx), ptr(self.midx), ptr(self.phfix),
                            ptr(self.model), ptr(self.info)), "gs_prefix")
        info = self.info.cpu().numpy()
        if info.any():
            raise np.linalg.LinAlgError(f"fixed-prior block not positive definite: info={info}")

    def tnt_host(self, p):
        m = int(self.m[p])
        o = int(self.tnt_off[p])
        return (self.TNT[o:o + m * m].view(m, m).cpu().numpy(),
                self.d[int(self.d_off[p]):int(self.d_off[p]) + m].cpu().numpy())

    # ------------------------------------------------------------------ b | rho
    def bdraw(self, phiinv_F, n_chain, z=None, sweep=0, event=_lib.EV_B, chain_base=0, out=None,
              info=None):
        """Batched b|rho: phiinv_F (P*n_chain, NF) device tensor -> b (P*n_chain, ldb)."""
        dev = self.ctx.device
        n_sys = self.P * n_chain
        b = out if out is not None else torch.zeros(n_sys, self.ldb, dtype=torch.float64, device=dev)
        inf = info if info is not None else torch.zeros(n_sys, dtype=torch.int32, device=dev)
        check(self.ctx.lib.gs_bdraw(self.ctx.handle, self.P, n_chain, self.NF, self.NMX, self.ldb,
                                    ptr(self.model), ptr(self.fidx), ptr(self.midx), ptr(self.nm_dev),
                                    ptr(phiinv_F), ptr(z), sweep, event, chain_base, ptr(b), ptr(inf)),
              "gs_bdraw")
        return b, inf


class FreeSpectrumChains:
    """n_chain independent free-spectrum Gibbs chains for each pulsar of a DeviceModel.

    State (HBM): x (P*n_chain, n_f) log10 rho, b (P*n_chain, ldb).
    ``run`` executes ``n_sweeps`` iterations of PulsarBlockGibbs.sample's loop
    body (pulsar_gibbs.py:656-698) in one persistent launch.
    """

    def __init__(self, model: DeviceModel, rhomin, rhomax, n_chain, x0, chain_base=0):
        self.model = model
        self.ctx = model.ctx
        self.n_chain = int(n_chain)
        self.rhomin, self.rhomax = float(rhomin), float(rhomax)
        self.chain_base = int(chain_base)
        self.n_f = model.NF // 2
        dev = self.ctx.device
        n_sys = model.P * self.n_chain
        x0 = np.broadcast_to(np.asarray(x0, float), (n_sys, self.n_f))
        self.x = _t(x0, torch.float64, dev)
        self.b = torch.zeros(n_sys, model.ldb, dtype=torch.float64, device=dev)
        self.info = torch.zeros(n_sys, dtype=torch.int32, device=dev)
        self.it = 0

    @property
    def n_sys(self):
        return self.model.P * self.n_chain

    def run(self, n_sweeps, record=True, record_b=True, z0_inj=None, z_inj=None, u_inj=None,
            x_rec=None, b_rec=None):
        m = self.model
        dev = self.ctx.device
        if record and x_rec is None:
            x_rec = torch.empty(n_sweeps, self.n_sys, self.n_f, dtype=torch.float64, device=dev)
        if record and record_b and b_rec is None:
            b_rec = torch.empty(n_sweeps, self.n_sys, m.ldb, dtype=torch.float64, device=dev)
        check(self.ctx.lib.gs_sweep_freespec(
            self.ctx.handle, m.P, self.n_chain, m.NF, m.NMX, m.ldb, ptr(m.model), ptr(m.fidx),
            ptr(m.midx), ptr(m.nm_dev), self.rhomin, self.rhomax, self.chain_base, ptr(self.x),
            ptr(self.b), self.it, int(n_sweeps), ptr(x_rec), ptr(b_rec), ptr(z0_inj), ptr(z_inj),
            ptr(u_inj), ptr(self.info)), "gs_sweep_freespec")
        self.it += int(n_sweeps)
        return x_rec, b_rec
