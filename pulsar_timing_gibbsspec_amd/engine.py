"""Device-resident state for the Gibbs hot path (HBM layout).

* ``DeviceModel`` — per-pulsar TNT/d (gs_tnt) and the fixed-prior Cholesky
  prefix (gs_prefix), built once from the PTA's T, N, r (the reference
  recomputes TNT/d every sweep, pulsar_gibbs.py:664-665; N is fixed in
  configs 1-4 so the result is identical).
* ``FreeSpectrumChains`` — n_chain independent chains per pulsar running the
  fused sweep kernel (gs_sweep_freespec): configs 1-3.
"""
from __future__ import annotations

import os

import numpy as np
import torch

from . import _lib
from ._lib import check, ptr

TUNED_NF = (20, 40, 60)          # fixed-NF instantiations (every broadcast variant)
FUSED_NF_MAX = 64                # register-tile b-draw and the fused sweep: any even NF <= 64
BIG_NF = (66, 254)               # even NF in this range: workspace-tile b-draw (config 5)
NMX_MAX = 128                    # fixed-prior (timing-model) columns per pulsar (> 64: NF <= 64,
NMX_FUSED = 64                   # gs_bdraw's wide kernel; the fused sweep keeps <= 64)


def nf_supported(NF):
    """NF = 2 n_f the b-draw handles (gs_bdraw, gs_bdraw_sys): any even NF <= 254."""
    return 0 < NF <= BIG_NF[1] and NF % 2 == 0


def _t(a, dtype, device):
    a = np.ascontiguousarray(a)
    if not a.flags.writeable:          # torch.as_tensor warns on read-only numpy buffers
        a = a.copy()
    return torch.as_tensor(a, dtype=dtype).to(device)


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
        if not nf_supported(NF):
            raise NotImplementedError(f"NF = 2*n_f = {NF}; supported: even NF <= {BIG_NF[1]}")
        self.P, self.NF = P, NF
        self.m = np.array([t.shape[1] for t in T_list], np.int64)
        self.n_toa = np.array([t.shape[0] for t in T_list], np.int64)
        self.nm = (self.m - NF).astype(np.int32)
        if (self.nm < 0).any() or (self.nm > NMX_MAX).any():
            raise NotImplementedError(f"need 0..{NMX_MAX} fixed-prior (timing-model) columns per pulsar")
        self.NMX = int(self.nm.max())
        if self.NMX > NMX_FUSED and NF > FUSED_NF_MAX:
            raise NotImplementedError(f"more than {NMX_FUSED} timing-model columns with NF > {FUSED_NF_MAX}")
        self.ldb = max(int(self.m.max()), NF + 1)    # the C-ABI wants ldb > NF (nm = 0 models)
        self.fidx_host = [np.asarray(f, np.int64) for f in fidx_list]
        self.midx_host = []
        fidx = np.zeros((P, NF), np.int32)
        # nm = 0 (MarginalizingTimingModel: no timing-model columns in T): the arrays keep
        # one (unused) column so their device pointers are not NULL
        midx = np.zeros((P, max(1, self.NMX)), np.int32)
        phfix = np.ones((P, max(1, self.NMX)))
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
        # TNT / d as double-double pairs (gs_tnt_dd -> gs_prefix_dd)
        self.TNT = torch.empty(int(np.sum(self.m * self.m)), dtype=torch.float64, device=dev)
        self.TNT_lo = torch.empty_like(self.TNT)
        self.d = torch.empty(int(np.sum(self.m)), dtype=torch.float64, device=dev)
        self.d_lo = torch.empty_like(self.d)
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
        self._lnl_const = None
        if Nvec is not None:
            self.Nvec.copy_(_t(np.concatenate(Nvec), torch.float64, self.ctx.device))
        lib, h = self.ctx.lib, self.ctx.handle
        check(lib.gs_tnt_dd(h, self.P, int(self.m.max()), ptr(self.tnt_desc), ptr(self.T), ptr(self.Nvec),
                            ptr(self.r), ptr(self.TNT), ptr(self.TNT_lo), ptr(self.d), ptr(self.d_lo)), "gs_tnt_dd")
        self.prefix()

    def prefix(self):
        """gs_prefix_dd of the resident (TNT, TNT_lo, d, d_lo): the model blocks and info."""
        lib, h = self.ctx.lib, self.ctx.handle
        check(lib.gs_prefix_dd(h, self.P, 1, self.NF, self.NMX, ptr(self.prefix_desc), 0, 0, ptr(self.TNT),
                               ptr(self.TNT_lo), ptr(self.d), ptr(self.d_lo), ptr(self.fidx), ptr(self.midx),
                               ptr(self.phfix), ptr(self.model), ptr(self.info)), "gs_prefix_dd")
        info = self.info.cpu().numpy()
        if info.any():
            raise np.linalg.LinAlgError(f"fixed-prior block not positive definite: info={info}")
        # register-tile copies for the one-draw-per-system b|rho launches (gs_bdraw_tiled)
        if self.NF <= FUSED_NF_MAX and self.NMX <= NMX_FUSED:
            ts = int(lib.gs_model_tiled_stride(self.NF, self.NMX))
            if getattr(self, "model_tiled", None) is None:
                self.model_tiled = torch.empty(self.P * ts, dtype=torch.float64, device=self.ctx.device)
            check(lib.gs_model_tile(h, self.P, self.NF, self.NMX, ptr(self.model), ptr(self.nm_dev),
                                    ptr(self.model_tiled)), "gs_model_tile")
        else:
            self.model_tiled = None

    def lnl_constants(self):
        """-1/2 (sum log N + r^T N^-1 r) + 1/2 sum_M log phiinv_M per pulsar (the model
        part of get_lnlikelihood_fullmarg, pulsar_gibbs.py:583-600), reduced on device."""
        if getattr(self, "_lnl_const", None) is not None:
            return self._lnl_const
        dev = self.ctx.device
        seg = torch.repeat_interleave(torch.arange(self.P, device=dev),
                                      torch.as_tensor(self.n_toa, device=dev))
        t = torch.log(self.Nvec) + self.r * self.r / self.Nvec
        wn = torch.zeros(self.P, dtype=torch.float64, device=dev).index_add_(0, seg, t)
        nmask = torch.arange(self.NMX, device=dev)[None, :] < self.nm_dev[:, None]
        lph = torch.where(nmask, torch.log(self.phfix), torch.zeros_like(self.phfix)).sum(dim=1)
        self._lnl_const = -0.5 * wn + 0.5 * lph
        return self._lnl_const

    def lnlike_marg(self, phiinv_F, n_chain):
        """Marginalised likelihood (pulsar_gibbs.py:569-610) of P*n_chain systems:
        phiinv_F (P*n_chain, NF) device tensor -> (lnl (P*n_chain,), info)."""
        dev = self.ctx.device
        n_sys = self.P * n_chain
        lnl = torch.empty(n_sys, dtype=torch.float64, device=dev)
        info = torch.zeros(n_sys, dtype=torch.int32, device=dev)
        check(self.ctx.lib.gs_lnlike_marg(self.ctx.handle, self.P, n_chain, self.NF, self.NMX, ptr(self.model), 0,
                                          ptr(self.nm_dev), ptr(phiinv_F), ptr(lnl), ptr(info)), "gs_lnlike_marg")
        const = self.lnl_constants().repeat_interleave(n_chain)
        return lnl + const, info

    def tnt_host(self, p):
        m = int(self.m[p])
        o = int(self.tnt_off[p])
        return (self.TNT[o:o + m * m].view(m, m).cpu().numpy(),
                self.d[int(self.d_off[p]):int(self.d_off[p]) + m].cpu().numpy())

    # ------------------------------------------------------------------ b | rho
    def bdraw(self, phiinv_F, n_chain, z=None, sweep=0, event=_lib.EV_B, chain_base=0, out=None,
              info=None, chain_mask=None):
        """Batched b|rho: phiinv_F (P*n_chain, NF) device tensor -> b (P*n_chain, ldb)."""
        dev = self.ctx.device
        n_sys = self.P * n_chain
        b = out if out is not None else torch.zeros(n_sys, self.ldb, dtype=torch.float64, device=dev)
        inf = info if info is not None else torch.zeros(n_sys, dtype=torch.int32, device=dev)
        check(self.ctx.lib.gs_bdraw(self.ctx.handle, self.P, n_chain, self.NF, self.NMX, self.ldb,
                                    ptr(self.model), ptr(self.fidx), ptr(self.midx), ptr(self.nm_dev),
                                    ptr(phiinv_F), ptr(z), sweep, event, chain_base, ptr(chain_mask),
                                    ptr(b), ptr(inf)),
              "gs_bdraw")
        return b, inf


class fail_counts:
    """Attach a per-system failed-draw counter (int32 device tensor) to the context for the
    duration of a block of launches (gs_ctx_set_fail_counts); the previous attachment is
    restored on exit (contexts are shared between engines, and scopes may nest).  The
    context's current attachment is tracked on the Python Context object."""

    def __init__(self, ctx, counts):
        self.ctx, self.counts = ctx, counts
        self._prev = None

    def __enter__(self):
        self._prev = getattr(self.ctx, "_fail_counts_attached", None)
        check(self.ctx.lib.gs_ctx_set_fail_counts(self.ctx.handle, ptr(self.counts)), "gs_ctx_set_fail_counts")
        self.ctx._fail_counts_attached = self.counts
        return self.counts

    def __exit__(self, *exc):
        check(self.ctx.lib.gs_ctx_set_fail_counts(self.ctx.handle, ptr(self._prev)), "gs_ctx_set_fail_counts")
        self.ctx._fail_counts_attached = self._prev
        return False


def check_handoff(info):
    """Raise if a fused-sweep chain was marked failed by the hand-off workgroups (info = -1:
    the bounded wait for the trio's previous third expired, so the chain's remaining sweeps
    were skipped instead of continuing from a stale slot).  Syncs."""
    bad = torch.nonzero(info < 0).flatten()
    if bad.numel():
        raise RuntimeError(f"fused sweep: {bad.numel()} chain(s) lost their hand-off (systems "
                           f"{bad[:8].tolist()}): their state was not advanced")


class FreeSpectrumChains:
    """n_chain independent free-spectrum Gibbs chains for each pulsar of a DeviceModel.

    State (HBM): x (P*n_chain, n_f) log10 rho, b (P*n_chain, ldb).
    ``run`` executes ``n_sweeps`` iterations of PulsarBlockGibbs.sample's loop
    body (pulsar_gibbs.py:656-698) in one persistent launch.
    """

    def __init__(self, model: DeviceModel, rhomin, rhomax, n_chain, x0, chain_base=0):
        self.fused = model.NF <= FUSED_NF_MAX and model.NMX <= NMX_FUSED
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
        # failed (non-PD) draws per system: the kernels keep b and count (gs_ctx_set_fail_counts)
        self.fail_count = torch.zeros(n_sys, dtype=torch.int32, device=dev)
        self.it = 0
        if not self.fused:
            self.xlast = torch.empty(n_sys, dtype=torch.float64, device=dev)
            self.gate = torch.ones(n_sys, dtype=torch.int32, device=dev)
            self.phiinv_F = torch.empty(n_sys, model.NF, dtype=torch.float64, device=dev)
            self.gw_col = torch.arange(self.n_f, dtype=torch.int32, device=dev)

    @property
    def n_sys(self):
        return self.model.P * self.n_chain

    def check_info(self):
        """Raise if any chain was marked failed by the hand-off workgroups (check_handoff)."""
        check_handoff(self.info)

    def run(self, n_sweeps, record=True, record_b=True, z0_inj=None, z_inj=None, u_inj=None,
            x_rec=None, b_rec=None, record_b_chains=None):
        """record_b_chains=K (< n_chain): b_rec holds only chains c < K of each pulsar, row
        sweep * P * K + p * K + c (GS_OPT_BREC_CHAINS) -- the reference's bchain is chain 0."""
        m = self.model
        dev = self.ctx.device
        bk = self.n_chain if record_b_chains is None else min(int(record_b_chains), self.n_chain)
        if record and x_rec is None:
            x_rec = torch.empty(n_sweeps, self.n_sys, self.n_f, dtype=torch.float64, device=dev)
        if record and record_b and b_rec is None:
            b_rec = torch.empty(n_sweeps, m.P * bk, m.ldb, dtype=torch.float64, device=dev)
        with fail_counts(self.ctx, self.fail_count):
            if not self.fused:
                self._run_sequence(n_sweeps, x_rec, b_rec if record_b else None, z0_inj, z_inj, u_inj, bk)
                return x_rec, b_rec
            self._run_fused(n_sweeps, x_rec, b_rec, z0_inj, z_inj, u_inj, bk)
        return x_rec, b_rec

    def _run_fused(self, n_sweeps, x_rec, b_rec, z0_inj, z_inj, u_inj, bk):
        m = self.model
        lib, h = self.ctx.lib, self.ctx.handle
        prev = self.ctx.get_option(_lib.OPT_BREC_CHAINS)
        self.ctx.set_option(_lib.OPT_BREC_CHAINS, bk if bk < self.n_chain else 0)
        try:
            check(lib.gs_sweep_freespec(
                h, m.P, self.n_chain, m.NF, m.NMX, m.ldb, ptr(m.model), ptr(m.fidx),
                ptr(m.midx), ptr(m.nm_dev), self.rhomin, self.rhomax, self.chain_base, ptr(self.x),
                ptr(self.b), self.it, int(n_sweeps), ptr(x_rec), ptr(b_rec), ptr(z0_inj), ptr(z_inj),
                ptr(u_inj), ptr(self.info)), "gs_sweep_freespec")
        finally:
            self.ctx.set_option(_lib.OPT_BREC_CHAINS, prev)
        self.it += int(n_sweeps)

    def _gate_phiinv(self, with_gate):
        check(self.ctx.lib.gs_pta_gate_phiinv(
            self.ctx.handle, 1, self.n_sys, self.n_f, self.n_f, ptr(self.x),
            ptr(self.xlast) if with_gate else None, ptr(self.gw_col), None, ptr(self.phiinv_F),
            ptr(self.gate)), "gs_pta_gate_phiinv")

    def _bdraw(self, z, event, mask):
        """gs_bdraw of every (pulsar, chain) system with the gate indexed by system."""
        m, lib, h = self.model, self.ctx.lib, self.ctx.handle
        per_sys = self.ctx.get_option(_lib.OPT_X_PER_SYS)
        self.ctx.set_option(_lib.OPT_X_PER_SYS, 1)
        inf = torch.zeros(self.n_sys, dtype=torch.int32, device=self.ctx.device)
        try:
            check(lib.gs_bdraw(h, m.P, self.n_chain, m.NF, m.NMX, m.ldb, ptr(m.model), ptr(m.fidx), ptr(m.midx),
                               ptr(m.nm_dev), ptr(self.phiinv_F), ptr(z), self.it, event, self.chain_base,
                               ptr(mask), ptr(self.b), ptr(inf)), "gs_bdraw")
        finally:
            self.ctx.set_option(_lib.OPT_X_PER_SYS, per_sys)
        torch.where(self.info == 0, inf, self.info, out=self.info)

    def _run_sequence(self, n_sweeps, x_rec, b_rec, z0_inj, z_inj, u_inj, bk=None):
        """NF > 64 (workspace-tile b draw): the same loop body as the fused kernel as a launch
        sequence per sweep -- record, [first draw], analytic rho|b (gs_rho_analytic), gate +
        phiinv, gated b|rho (gs_bdraw) -- with the same Philox counters per draw."""
        m, lib, h = self.model, self.ctx.lib, self.ctx.handle
        for i in range(int(n_sweeps)):
            ii = self.it
            check(lib.gs_pta_record(h, self.n_sys, self.n_f, ptr(self.x), ptr(x_rec[i]) if x_rec is not None
                                    else None, ptr(self.xlast)), "gs_pta_record")   # pulsar_gibbs.py:658
            if b_rec is not None:                                                    # :659
                if bk is None or bk >= self.n_chain:
                    b_rec[i].copy_(self.b)
                else:
                    b_rec[i].copy_(self.b.view(m.P, self.n_chain, m.ldb)[:, :bk].reshape(m.P * bk, m.ldb))
            if ii == 0:                                                              # :661-662
                self._gate_phiinv(with_gate=False)
                self._bdraw(z0_inj, _lib.EV_B0, None)
            check(lib.gs_rho_analytic(h, m.P, self.n_chain, m.NF, m.ldb, ptr(m.fidx), ptr(self.b),
                                      ptr(u_inj[i]) if u_inj is not None else None, ii, self.chain_base,
                                      self.rhomin, self.rhomax, ptr(self.x), self.n_f), "gs_rho_analytic")
            self._gate_phiinv(with_gate=True)                                        # :697
            self._bdraw(z_inj[i] if z_inj is not None else None, _lib.EV_B, self.gate)   # :698
            self.it += 1


class HistoryStreamer:
    """Chain history to pinned host memory, overlapped with the sampling.

    Two slots of device record buffers; after a block of sweeps is launched on the
    context stream, ``submit`` queues its device->pinned-host copy on a side stream
    (ordered after the block by an event) and returns at once, so the copy runs on
    the copy engine while the next block's sweeps run.  ``fetch`` waits for a slot's
    copy and returns the pinned host tensors.  A slot is reused only after its fetch."""

    def __init__(self, ctx, shapes, dtype=torch.float64, views=None, direct=None):
        """shapes: device record buffers (rows first); views[i] (optional): the part of a
        block of buffer i that goes to the host, e.g. ``lambda t: t[:, ::nc]`` for chain 0
        of every pulsar -- the rest stays in HBM and never crosses PCIe.  direct[i] (no view):
        the kernels write buffer i straight into the pinned host slot (zero-copy): no copy
        and no staging in HBM.  Measured on MI355X for the configs[1] headline (x rows of
        4096 chains, 98 MB per 100 sweeps): 2.97 ms per 100-sweep block written straight
        to the host vs 2.73 ms into HBM and 4.2 ms with the copy overlapped on a side stream
        (tools/stream_probe.py)."""
        dev = ctx.device
        self.ctx = ctx
        n = len(shapes)
        self.views = list(views) if views is not None else [None] * n
        self.direct = [bool(d) and v is None for d, v in zip(direct or [False] * n, self.views)]
        self.views = [v if v is not None else (lambda t: t) for v in self.views]
        hshapes = [tuple(v(torch.empty(s, device="meta")).shape) for s, v in zip(shapes, self.views)]
        self.host_bufs = [[torch.empty(s, dtype=dtype, pin_memory=True) for s in hshapes] for _ in range(2)]
        self.dev_bufs = [[h if d else torch.empty(s, dtype=dtype, device=dev)
                          for s, h, d in zip(shapes, hb, self.direct)] for hb in self.host_bufs]
        self.side = torch.cuda.Stream(device=dev)
        self.done = [torch.cuda.Event(), torch.cuda.Event()]
        self.rows = [0, 0]

    def buffers(self, slot, n):
        return [b[:n] for b in self.dev_bufs[slot]]

    def submit(self, slot, n):
        ready = torch.cuda.Event()
        ready.record(self.ctx.stream)
        with torch.cuda.stream(self.side):
            self.side.wait_event(ready)
            for d, h, v, direct in zip(self.dev_bufs[slot], self.host_bufs[slot], self.views, self.direct):
                if not direct:
                    h[:n].copy_(v(d[:n]), non_blocking=True)
            self.done[slot].record(self.side)
        self.rows[slot] = n

    def fetch(self, slot):
        self.done[slot].synchronize()
        return [h[:self.rows[slot]] for h in self.host_bufs[slot]]


def grid3(rhomin, rhomax, n=1000, device="cuda"):
    """[rho_g | log rho_g | 0.5 log10 rho_g], rho_g = 10**linspace(log10 rhomin, log10 rhomax, n)
    — numpy on the host, so the device sees the reference's exact grid
    (pulsar_gibbs.py:228, pta_gibbs.py:189-190, 254-255)."""
    g = 10 ** np.linspace(np.log10(rhomin), np.log10(rhomax), n)
    return _t(np.concatenate([g, np.log(g), 0.5 * np.log10(g)]), torch.float64, device)


class PTAChains:
    """n_chain chains of the common free-spectrum model (CURN) over the pulsars of a
    DeviceModel, optionally with per-pulsar red free spectra drawn conditionally
    (PTABlockGibbs.sample, pta_gibbs.py:664-704).

    Per sweep (one host-side launch sequence, all chains at once):
      record x (row ii) -> [ii == 0: b|rho from x0] -> tau -> [red grid-CDF]
      -> [exchange] -> common grid-CDF -> gate + phiinv -> gated b|rho.
    State (HBM): x (n_chain, n_param) in the PTA's parameter order (every rank
    holds the full vector), b (P_local*n_chain, ldb).

    Pulsar sharding: the DeviceModel holds this rank's contiguous pulsar block
    [psr_lo, psr_lo + P_local) of P_global; ``gather`` (distributed.PulsarAllGather)
    exchanges the [tau | x_red] slabs so the common draw sees every pulsar in global
    order.  ``sweep_begin`` / ``sweep_end`` expose the two halves around the exchange.

    curn_mode='sum' (no per-pulsar red noise only): the common draw uses the sufficient
    statistic S_k = sum_p tau_p,k, summed exactly in fixed point (gs_tau_sum_fx ->
    gs_fx_to_double -> gs_rho_curn_sum); a pulsar-sharded run exchanges the int64 digits with
    ``allreduce`` (distributed.TauSumAllReduce, one RCCL all-reduce of 3 x n_f x n_chain int64 per
    sweep) instead of gathering tau, and reproduces the unsharded chains bit for bit for any
    number of shards.
    """

    def __init__(self, model: DeviceModel, n_param, gw_col, red_col, gw_bounds, red_bounds, n_chain, x0,
                 chain_base=0, ngrid=1000, P_global=None, psr_lo=0, gather=None, curn_mode="exact",
                 allreduce=None, hyper=None, hyper_acl=None, hyper_warmup=None):
        """hyper (pta_hyper.HyperSpec): per-pulsar red noise sampled by the Metropolis block
        (PTABlockGibbs redsample='mh', pta_gibbs.py:278-340) instead of red_col's conditional
        grid draws; hyper_acl steps per sweep (None: estimated from sweep 0's hyper_warmup
        steps, pta_hyper.hyper_aclength)."""
        self.model, self.ctx = model, model.ctx
        dev = self.ctx.device
        P, C = model.P, int(n_chain)
        self.P, self.C, self.n_param = P, C, int(n_param)
        self.PG = int(P_global) if P_global is not None else P
        self.psr_lo = int(psr_lo)
        if hyper is not None:
            if red_col is not None:
                raise ValueError("give either red_col (conditional red draws) or hyper (Metropolis), not both")
            if hyper.P != self.PG:
                raise ValueError(f"the hyper tables cover {hyper.P} pulsars, the array {self.PG}")
            if hyper.kind == 0:
                red_col = hyper.red_col_host           # the free-spectrum red columns (irn, phiinv)
        # the exchange runs when pulsars are split over ranks, or whenever one is given (a
        # 1-rank group exercises the same launch sequence, e.g. to capture it in a graph)
        self.sharded = self.PG != P or (allreduce if curn_mode == "sum" else gather) is not None
        self.gather = gather
        if curn_mode not in ("exact", "sum"):
            raise ValueError("curn_mode must be 'exact' or 'sum'")
        if curn_mode == "sum" and (red_col is not None or hyper is not None):
            raise ValueError("curn_mode='sum' needs irn = 0 (no per-pulsar red noise)")
        self.curn_mode = curn_mode
        self.allreduce = allreduce
        if self.sharded and curn_mode == "exact" and gather is None:
            raise ValueError("a pulsar-sharded PTAChains needs a gather")
        if self.sharded and curn_mode == "sum" and allreduce is None:
            raise ValueError("a pulsar-sharded curn_mode='sum' PTAChains needs an allreduce")
        self.n_f = model.NF // 2
        self.chain_base = int(chain_base)
        self.ngrid = ngrid
        self.ctx.set_option(_lib.OPT_PSR_BASE, self.psr_lo)
        self.gw_col = _t(np.asarray(gw_col, np.int32), torch.int32, dev)
        self.hyper_spec = hyper
        self.hyper_pl = hyper is not None and hyper.kind == 1       # power-law red phi (gs_phi_powerlaw)
        # self.red: per-pulsar red noise in phi (irn in the common draw); red_cond: drawn by the grid
        # conditional (redsample='conditional'); otherwise by the hyper MH block
        self.red = red_col is not None or self.hyper_pl
        self.red_cond = red_col is not None and hyper is None
        if red_col is not None:
            rg = np.asarray(red_col, np.int32).reshape(self.PG, self.n_f)
            self.red_col_g = _t(rg.ravel(), torch.int32, dev)
            self.red_col = _t(rg[self.psr_lo:self.psr_lo + P].ravel(), torch.int32, dev)
        else:
            self.red_col = self.red_col_g = None
        # the x columns of each pulsar's red parameters [PG x W] -- what a pulsar-sharded run exchanges
        # besides tau (a rank draws only its own pulsars' red parameters): the red free spectrum
        # (W = n_f) or the power law's (log10_A, gamma) (W = 2)
        xred = None
        if self.hyper_pl:
            xred = np.asarray(hyper.pl_col_host, np.int64).reshape(self.PG, -1)
        elif red_col is not None:
            xred = np.asarray(red_col, np.int64).reshape(self.PG, self.n_f)
        self.xred_w = 0 if xred is None else xred.shape[1]
        self.xred_rows = -(-self.xred_w // self.n_f)          # slab rows the red x values take
        if xred is not None:
            self.xred_l64 = torch.as_tensor(xred[self.psr_lo:self.psr_lo + P].ravel(), dtype=torch.long, device=dev)
            self.xred_g64 = torch.as_tensor(xred.ravel(), dtype=torch.long, device=dev)
        self.grid_gw = grid3(*gw_bounds, n=ngrid, device=dev)
        self.grid_red = grid3(*red_bounds, n=ngrid, device=dev) if self.red_cond else None
        self.x = _t(np.broadcast_to(np.asarray(x0, float), (C, self.n_param)), torch.float64, dev)
        self.b = torch.zeros(P * C, model.ldb, dtype=torch.float64, device=dev)
        self.tau = torch.empty(P, self.n_f, C, dtype=torch.float64, device=dev)
        self.tau_g = torch.empty(self.PG, self.n_f, C, dtype=torch.float64, device=dev) if self.sharded \
            else self.tau
        self.S = torch.empty(self.n_f, C, dtype=torch.float64, device=dev)   # curn_mode='sum'
        # ... as exact fixed-point digits (gs_tau_sum_fx): the exchanged quantity of a sharded run,
        # order-free, so every shard count gives the 1-shard S bit for bit
        self.S_fx = torch.empty(3, self.n_f, C, dtype=torch.int64, device=dev)
        self.fx_e0 = int(np.floor(np.log2(gw_bounds[0]))) - 64
        self.fx_ovf = torch.zeros(1, dtype=torch.int32, device=dev)
        self.gwphi = torch.empty(self.n_f, C, dtype=torch.float64, device=dev)
        self.irn = torch.empty(self.PG, self.n_f, C, dtype=torch.float64, device=dev) if self.red else None
        # without per-pulsar red noise phiinv is the common spectrum alone, the same for every
        # pulsar: one row per chain (GS_OPT_PHI_PER_CHAIN) instead of P rows of it
        self.phi_shared = not self.red
        self.phiinv_F = torch.empty((1 if self.phi_shared else P) * C, model.NF, dtype=torch.float64, device=dev)
        self.gate = torch.ones(C, dtype=torch.int32, device=dev)
        self.xlast = torch.empty(C, dtype=torch.float64, device=dev)
        self.info = torch.zeros(P * C, dtype=torch.int32, device=dev)
        self.fail_count = torch.zeros(P * C, dtype=torch.int32, device=dev)   # failed draws (b kept)
        self.slab_shape = (1 + self.xred_rows, self.n_f, C)
        self.it = 0
        self.redraw_b = False      # draw b | x first at the next sweep, as at sweep 0 (resume)
        self.hyper = None
        if hyper is not None:
            from .pta_hyper import HYPER_WARMUP, HyperMH
            self.hyper = HyperMH(hyper, model, C, self.n_param, self.gw_col, psr_lo=self.psr_lo)
            self.hyper_acl = None if hyper_acl is None else int(hyper_acl)
            self.hyper_warmup = HYPER_WARMUP if hyper_warmup is None else int(hyper_warmup)
            self.hyper_short_chain = None      # chain 0's sweep-0 warm-up proposals (q[hind] rows)
            # phiinv of every (pulsar, chain) at the block's start (seeds lnL_p), separate from the
            # b draw's rows so the gate's phiinv is untouched
            self.phiinv_h = torch.empty(P * C, model.NF, dtype=torch.float64, device=dev)
            self._gate_h = torch.empty(C, dtype=torch.int32, device=dev)

    def _bdraw(self, z, event, mask):
        m, lib, h = self.model, self.ctx.lib, self.ctx.handle
        prev = self.ctx.get_option(_lib.OPT_PHI_PER_CHAIN)
        self.ctx.set_option(_lib.OPT_PHI_PER_CHAIN, int(self.phi_shared))
        # the register-tile copies of the model blocks when the tile variant is selected (the default)
        tiled = (m.model_tiled is not None and self.ctx.get_option(_lib.OPT_BCAST) == 3
                 and os.environ.get("GS_PTA_TILED", "1") != "0")        # A/B knob
        fn, name = (lib.gs_bdraw_tiled, "gs_bdraw_tiled") if tiled else (lib.gs_bdraw, "gs_bdraw")
        # the red MH block's lnL_p seed as a by-product of the draw (gs_ctx_set_bdraw_lnl): the draw
        # factorises every (pulsar, chain) system at the phiinv the next block starts from, and the
        # systems a gated draw skips get the likelihood-mode factorisation in the same launch
        # (pta_gibbs.py:689-704 order)
        lnl = self.hyper is not None and tiled and not self.phi_shared
        if lnl:
            check(lib.gs_ctx_set_bdraw_lnl(h, ptr(self.hyper.lnl_p), ptr(m.model)), "gs_ctx_set_bdraw_lnl")
        try:
            check(fn(h, m.P, self.C, m.NF, m.NMX, m.ldb, ptr(m.model_tiled if tiled else m.model), ptr(m.fidx),
                     ptr(m.midx), ptr(m.nm_dev), ptr(self.phiinv_F), ptr(z), self.it, event, self.chain_base,
                     ptr(mask), ptr(self.b), ptr(self.info)), name)
        finally:
            self.ctx.set_option(_lib.OPT_PHI_PER_CHAIN, prev)
            if lnl:
                check(lib.gs_ctx_set_bdraw_lnl(h, None, None), "gs_ctx_set_bdraw_lnl")
        if lnl:
            self.hyper.fresh = True

    def _gate_phiinv(self, with_gate, out=None, gate=None):
        out = self.phiinv_F if out is None else out
        gate = self.gate if gate is None else gate
        if self.hyper_pl or self.red_cond:
            # phi = 10^(2 x_gw) + irn, irn current with x: the power-law red phi, or the red free
            # spectrum's 10^(2 x_red) that gs_phi_from_x already formed for the common draw (the
            # same pow: the same bits as recomputing it per (pulsar, bin) here)
            irn = self.irn[self.psr_lo:self.psr_lo + self.P]
            check(self.ctx.lib.gs_pta_gate_phiinv_irn(
                self.ctx.handle, self.P, self.C, self.n_f, self.n_param, ptr(self.x),
                ptr(self.xlast) if with_gate else None, ptr(self.gw_col), ptr(irn), ptr(out),
                ptr(gate)), "gs_pta_gate_phiinv_irn")
            return
        check(self.ctx.lib.gs_pta_gate_phiinv(
            self.ctx.handle, 1 if self.phi_shared else self.P, self.C, self.n_f, self.n_param, ptr(self.x),
            ptr(self.xlast) if with_gate else None, ptr(self.gw_col), ptr(self.red_col),
            ptr(out), ptr(gate)), "gs_pta_gate_phiinv")

    def _update_irn(self):
        """Per-pulsar red phi at the current x (the common draw's irn, pta_gibbs.py:197-198)."""
        if self.hyper_pl:
            self.hyper.irn(self.x, self.irn)
        elif self.red:
            check(self.ctx.lib.gs_phi_from_x(self.ctx.handle, self.C, self.PG * self.n_f, ptr(self.x), self.n_param,
                                             ptr(self.red_col_g), ptr(self.irn)), "gs_phi_from_x")

    def hyper_block(self, nsteps, inj=None, q_rec=None, seed=True):
        """The red hyper-parameter Metropolis block (pta_gibbs.py:278-340) for every chain:
        lnL_p of every (pulsar, chain) seeded at the current x (seed=False: lnl_p is already that,
        from the last b draw), then nsteps steps in place."""
        h = self.hyper
        if seed:
            if self.hyper_pl:
                self._update_irn()
            self._gate_phiinv(with_gate=False, out=self.phiinv_h, gate=self._gate_h)
            h.seed(self.phiinv_h)
        h.steps(self.x, nsteps, self.it, self.chain_base, inj=inj, q_rec=q_rec)
        h.fresh = False

    def sweep_begin(self, x_rec=None, z0=None, u_red=None, mh_inj=None):
        """Record, [first draw], [hyper MH], tau and the local red draws.  Returns the local
        exchange slab [P_local, 1 or 2, n_f, C] (None when not sharded)."""
        lib, h, m = self.ctx.lib, self.ctx.handle, self.model
        ii = self.it
        check(lib.gs_pta_record(h, self.C, self.n_param, ptr(self.x), ptr(x_rec), ptr(self.xlast)),
              "gs_pta_record")
        if ii == 0 or self.redraw_b:                           # pta_gibbs.py:669-670
            if self.hyper_pl or self.red_cond:
                self._update_irn()
            self._gate_phiinv(with_gate=False)
            self._bdraw(z0, _lib.EV_B0, None)
            self.redraw_b = False
        if self.hyper is not None:                             # pta_gibbs.py:689-697 (redsample='mh')
            if ii == 0:
                n = self.hyper_warmup
                # zeroed: a pulsar-sharded rank records only the steps of its own pulsars, and the
                # ranks' records are summed below (every step is owned by exactly one rank)
                q_rec = torch.zeros(n, self.C, 3, dtype=torch.float64, device=self.ctx.device) \
                    if self.hyper_acl is None else None
                x_start = self.x[0].cpu().numpy() if q_rec is not None else None
                self.hyper_block(n, inj=mh_inj, q_rec=q_rec, seed=not self.hyper.fresh)
                if q_rec is not None:                          # aclength_hyper from the warm-up (:311-315)
                    from .pta_hyper import hyper_aclength
                    q0 = q_rec[:, 0].contiguous()
                    if self.sharded:
                        from .distributed import allreduce_sum
                        q0 = allreduce_sum(q0, group=getattr(self.gather, "group", None))
                    self.hyper_short_chain = self.hyper_spec.short_chain(x_start, q0.cpu().numpy())
                    self.hyper_acl = hyper_aclength(self.hyper_short_chain)
            else:
                self.hyper_block(self.hyper_acl, inj=mh_inj, seed=not self.hyper.fresh)
        if self.curn_mode == "sum":                            # sufficient statistic S_k
            # tau and its fixed-point digits in one pass over b (tau itself is not needed)
            check(lib.gs_tau_sum_fx_b(h, self.P, self.C, m.NF, m.ldb, ptr(m.fidx), ptr(self.b), self.fx_e0,
                                      ptr(self.S_fx), ptr(self.fx_ovf)), "gs_tau_sum_fx_b")
            return self.S_fx if self.sharded else None
        check(lib.gs_tau(h, self.P, self.C, m.NF, m.ldb, ptr(m.fidx), ptr(self.b), 0, ptr(self.tau)),
              "gs_tau")
        if self.red_cond:                                      # pta_gibbs.py:252-276
            check(lib.gs_phi_from_x(h, self.C, self.n_f, ptr(self.x), self.n_param, ptr(self.gw_col),
                                    ptr(self.gwphi)), "gs_phi_from_x")
            check(lib.gs_rho_red(h, self.P, self.C, self.n_f, ptr(self.tau), ptr(self.gwphi), self.ngrid,
                                 ptr(self.grid_red), ptr(u_red), ii, self.chain_base, ptr(self.x),
                                 self.n_param, ptr(self.red_col), None), "gs_rho_red")
        if not self.sharded:
            return None
        slab = torch.zeros((self.P,) + self.slab_shape, dtype=torch.float64, device=self.ctx.device)
        slab[:, 0] = self.tau
        if self.xred_w:
            xr = self.x.index_select(1, self.xred_l64).T.reshape(self.P, self.xred_w, self.C)
            slab[:, 1:].view(self.P, self.xred_rows * self.n_f, self.C)[:, :self.xred_w] = xr
        return slab

    def sweep_end(self, slab_g=None, z=None, u_curn=None):
        """Common draw on the global inputs, gate, gated b|rho."""
        lib, h = self.ctx.lib, self.ctx.handle
        ii = self.it
        if self.curn_mode == "sum":
            if self.sharded and slab_g is not None and slab_g.data_ptr() != self.S_fx.data_ptr():
                self.S_fx.copy_(slab_g)
            check(lib.gs_fx_to_double(h, self.n_f * self.C, self.fx_e0, ptr(self.S_fx), ptr(self.S)),
                  "gs_fx_to_double")
            check(lib.gs_rho_curn_sum(h, self.PG, self.C, self.n_f, ptr(self.S), self.ngrid, ptr(self.grid_gw),
                                      ptr(u_curn), ii, self.chain_base, ptr(self.x), self.n_param,
                                      ptr(self.gw_col), None), "gs_rho_curn_sum")
            self._gate_phiinv(with_gate=True)
            self._bdraw(z, _lib.EV_B, self.gate)
            self.it += 1
            return
        if self.sharded:
            self.tau_g.copy_(slab_g[:, 0])
            if self.xred_w:
                xr = slab_g[:, 1:].reshape(self.PG, self.xred_rows * self.n_f, self.C)[:, :self.xred_w]
                self.x.index_copy_(1, self.xred_g64, xr.reshape(self.PG * self.xred_w, self.C).T.contiguous())
        self._update_irn()
        check(lib.gs_rho_curn(h, self.PG, self.C, self.n_f, ptr(self.tau_g), ptr(self.irn), self.ngrid,
                              ptr(self.grid_gw), ptr(u_curn), ii, self.chain_base, ptr(self.x),
                              self.n_param, ptr(self.gw_col), None), "gs_rho_curn")   # pta_gibbs.py:181-214
        self._gate_phiinv(with_gate=True)                      # pta_gibbs.py:703
        self._bdraw(z, _lib.EV_B, self.gate)                   # pta_gibbs.py:704
        self.it += 1

    def hyper_acceptance(self):
        """Accepted fraction of the red MH steps per chain since the engine was built; a
        pulsar-sharded run sums the ranks' counts (each rank takes the steps of its own pulsars).
        Syncs."""
        if self.hyper is None:
            return None
        acc = self.hyper.acc_total.double()
        if self.sharded:
            from .distributed import allreduce_sum
            acc = allreduce_sum(acc.clone(), group=getattr(self.gather, "group", None))
        return (acc / max(1, self.hyper.steps_total)).cpu().numpy()

    def check_fx(self):
        """curn_mode='sum': raise if gs_tau_sum_fx_b saw a tau it cannot sum exactly (negative,
        non-finite or >= rhomin_gw * 2^80, the fixed-point window) since the engine was built:
        S would then be wrong.  Syncs."""
        if self.curn_mode == "sum" and int(self.fx_ovf.item()):
            raise RuntimeError("curn_mode='sum': a tau fell outside the fixed-point window (negative, "
                               "non-finite or >= rhomin_gw * 2**80); rerun with curn_mode='exact'")

    def capture(self, n_sweeps):
        """Capture n_sweeps steady-state sweeps (device Philox) into a hipGraph
        (torch.cuda.CUDAGraph around the C-ABI launches on the context's stream).

        Philox counters take sweep = launch argument + a device counter
        (gs_ctx_set_sweep_counter), which the graph advances itself (gs_counter_add),
        so every replay draws the next n_sweeps sweeps: replays are bit-identical to
        eager sweeps.  The graph records x into ``graph_rec`` (n_sweeps, C, n_param).

        A pulsar-sharded engine captures its per-sweep exchange too: the RCCL all-reduce of
        the fixed-point tau-sum digits (or the [tau | x_red] all-gather) is issued on the
        capture stream and becomes a node of the graph, so a replay runs n_sweeps sweeps with
        no return to the host.  That needs the 'nccl' (RCCL) backend; gloo collectives run on
        the host and cannot be captured."""
        if self.it == 0:
            raise ValueError("run sweep 0 eagerly first (it draws b from x0, pta_gibbs.py:669-670)")
        if self.sharded:
            import torch.distributed as dist
            if not dist.is_initialized() or dist.get_backend() != "nccl":
                raise NotImplementedError("graph capture of the pulsar-sharded exchange needs the 'nccl' "
                                          "(RCCL) backend; gloo collectives run on the host")
        lib, h, dev = self.ctx.lib, self.ctx.handle, self.ctx.device
        n = int(n_sweeps)
        self.graph_rec = torch.empty(n, self.C, self.n_param, dtype=torch.float64, device=dev)
        self._gcount = torch.zeros(1, dtype=torch.int64, device=dev)
        self._gbase, self._gn = self.it, n
        cap = torch.cuda.Stream(device=dev)
        old = self.ctx.stream
        cap.wait_stream(old)
        self.ctx.set_stream(cap)
        check(lib.gs_ctx_set_sweep_counter(h, ptr(self._gcount)), "gs_ctx_set_sweep_counter")
        self.graph = torch.cuda.CUDAGraph()
        # the hyper block's step count is host-side: nothing runs during capture, and each replay
        # adds the captured sweeps' steps (its accepted-step counter is a device add the graph replays)
        hsteps0 = self.hyper.steps_total if self.hyper is not None else 0
        try:
            with torch.cuda.graph(self.graph, stream=cap):
                for i in range(n):
                    self.sweep(x_rec=self.graph_rec[i])
                check(lib.gs_counter_add(h, ptr(self._gcount), n), "gs_counter_add")
        finally:
            check(lib.gs_ctx_set_sweep_counter(h, None), "gs_ctx_set_sweep_counter")
            self.ctx.set_stream(old)
            self.it = self._gbase          # nothing ran during capture
            if self.hyper is not None:
                self._g_hsteps = self.hyper.steps_total - hsteps0
                self.hyper.steps_total = hsteps0
        return self.graph_rec

    def replay(self):
        """Run the captured sweeps once (the next n_sweeps sweeps); returns graph_rec."""
        self._gcount.fill_(self.it - self._gbase)   # stays right if eager sweeps ran between
        self.graph.replay()
        self.it += self._gn
        if self.hyper is not None:
            self.hyper.steps_total += self._g_hsteps
        return self.graph_rec

    def sweep(self, x_rec=None, z0=None, z=None, u_red=None, u_curn=None, mh_inj=None):
        """One PTABlockGibbs sweep for every chain; x_rec: (n_chain, n_param) row or None.
        z0/z: (P*n_chain, ldb) injected normals (original column order); u_red
        (n_chain, P, n_f) and u_curn (n_chain, n_f): injected uniforms; mh_inj (steps, n_chain,
        4): injected hyper-MH draws (scale, j, randn, rand)."""
        with fail_counts(self.ctx, self.fail_count):
            slab = self.sweep_begin(x_rec=x_rec, z0=z0, u_red=u_red, mh_inj=mh_inj)
            if self.sharded:
                # the collective is ordered after the slab's kernels: torch issues it against the
                # CURRENT stream, which is made the context's (the kernels' stream; a no-op when the
                # context runs on torch's current stream, as by default and inside graph capture)
                with torch.cuda.stream(self.ctx.stream):
                    slab = self.allreduce(slab) if self.curn_mode == "sum" else self.gather(slab)
            self.sweep_end(slab, z=z, u_curn=u_curn)
