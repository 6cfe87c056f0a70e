"""Benchmark: Gibbs iterations/s (all chains, whole node) + ESS/s of log10 rho.

Workload (BASELINE.json configs[1]): the simulated J1713+0747 pulsar (720 TOAs,
30-bin free spectrum + 16-column timing model, m = 76, fixed white noise),
``--chains`` independent chains per GPU (default 4096), batched on each MI355X.
A "step" = one Gibbs sweep of every chain (rho|b then b|rho, with the chain
rows recorded to HBM as PulsarBlockGibbs.sample records them).

N GPUs: one process per GPU (torch.distributed.run), chains sharded by rank
(chain_base = rank * chains, disjoint Philox streams), no data-path collective
-> weak scaling.  Timing: barrier + synchronize on both sides of exactly K
steps, max over ranks.

Extra fields: "roofline" (fp64 work of the fused sweep kernel per launch over
its HIP-event-timed duration on the launch stream), "cpu_baseline" (the
oracle's restatement of the reference loop, numpy/LAPACK SVD, 1 thread, on this
host), "ess_per_s" (min over bins of the summed ESS/s).
"""
import argparse
import json
import os
import sys
import time

os.environ.setdefault("OPENBLAS_NUM_THREADS", "1")   # reference-faithful CPU baseline

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

FP64_PEAK_TFLOPS = 78.6          # MI355X FP64 vector = FP64 matrix, AMD public spec
HBM_PEAK_GBS = 8000.0


def flops_per_chain_sweep(m):
    """potrf m^3/3 + m^2/2 + m/6 + 3 triangular solves 3 m^2."""
    return m ** 3 / 3 + m ** 2 / 2 + m / 6 + 3 * m ** 2


def executed_flops_per_chain_sweep(nf, nm):
    """What the kernel executes (NF x NF Schur block + solves + fixed-prior GEMVs)."""
    return nf ** 3 / 3 + nf ** 2 / 2 + nf / 6 + 2 * nf ** 2 + 2 * nm * nf + nm ** 2


def pmc_traffic(S, C):
    """HBM bytes per launch of k_sweep_freespec from the committed PMC profile
    (tools/gpu_profile.sh -> tools/pmc_traffic.py), valid for the same launch shape."""
    f = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        d = json.load(open(f))
    except (OSError, ValueError):
        return None
    if d.get("sweeps_per_launch") != S or d.get("chains") != C or "bytes_per_launch" not in d:
        return None
    return d["bytes_per_launch"]


def cpu_baseline(seconds=12.0):
    """Reference loop (oracle restatement, SVD draw), 1 thread, bounded sample."""
    from oracle import gibbs_oracle as O
    from pulsar_timing_gibbsspec_amd import synthetic
    pta = synthetic.single_pulsar_pta("J1713+0747", seed=0)
    T, N, r = pta.get_basis()[0], pta.get_ndiag({})[0], pta.get_residuals()[0]
    gwid = np.arange(60)
    rng = np.random.default_rng(0)
    x = rng.uniform(-9, -4, 30)
    b = np.zeros(T.shape[1])
    n_tm = T.shape[1] - 60
    it = 0
    t0 = time.perf_counter()
    while True:
        TNT, d = O.tnt(T, N, r)                    # recomputed every sweep (pulsar_gibbs.py:664-665)
        if it == 0:                                # first draw from xs (pulsar_gibbs.py:661-662)
            b = O.bdraw_svd(TNT, d, O.phiinv_single(x, n_tm), rng.standard_normal(T.shape[1]))
        tau = O.tau_half(b, gwid)
        x = 0.5 * np.log10(O.rho_analytic(tau, rng.random(30), 1e-18, 1e-8))
        b = O.bdraw_svd(TNT, d, O.phiinv_single(x, n_tm), rng.standard_normal(T.shape[1]))
        it += 1
        el = time.perf_counter() - t0
        if el > seconds:
            break
    return dict(value=it / el, unit="iters/s", cores=1, kind="port",
                sample=f"{it} sweeps of the J1713 single-chain loop (oracle restatement of "
                       f"pulsar_gibbs.py:656-698, numpy/OpenBLAS SVD, OPENBLAS_NUM_THREADS=1) in {el:.1f} s")


def ess_min_bin(x_rec, elapsed, n_chains_total, max_chains=256):
    """Min over the 30 bins of the whole-job ESS/s of log10 rho.

    IAT per chain on the post-burn-in rows (first 20 % dropped) of up to
    ``max_chains`` chains; ESS/s = mean ESS per chain x all chains / the time
    the post-burn-in sweeps took."""
    from pulsar_timing_gibbsspec_amd.diagnostics import iat
    xr = x_rec[:, :max_chains]                      # (K, C, n_f)
    K, C, nf = xr.shape
    burn = K // 5
    n = K - burn
    ess = np.array([np.mean([n / max(iat(xr[burn:, c, k]), 1.0) for c in range(C)]) for k in range(nf)])
    return float(ess.min() * n_chains_total / (elapsed * n / K))


def pta_cpu_baseline(kind, seconds=10.0):
    """The oracle's restatement of PTABlockGibbs.sample (pta_gibbs.py:664-704), SVD draws,
    1 thread, bounded sample of the same 45-pulsar model."""
    from oracle import gibbs_oracle as O
    from pulsar_timing_gibbsspec_amd import synthetic
    pta = synthetic.array_pta(kind=kind, seed=0)
    T, N, R = pta.get_basis(), pta.get_ndiag({}), pta.get_residuals()
    P = len(T)
    TNT = [O.tnt(T[p], N[p], R[p]) for p in range(P)]
    names = pta.param_names
    rind = np.array([i for i, n in enumerate(names) if "rho" in n and "gw" in n])
    hind = np.array([i for i, n in enumerate(names) if "red" in n and "rho" in n])
    rng = np.random.default_rng(0)
    x = rng.uniform(-9, -4, len(names))
    m = [t.shape[1] for t in T]
    gw = [np.arange(mm - 60, mm) for mm in m]

    def draw(x):
        out = []
        for p in range(P):
            phi = 10 ** (2 * x[rind]) + (10 ** (2 * x[hind[p * 30:(p + 1) * 30]]) if kind == "curn_red" else 0)
            ph = np.full(m[p], 1e-40)
            ph[gw[p]] = 1 / np.repeat(phi, 2)
            out.append(O.bdraw_svd(TNT[p][0], TNT[p][1], ph, rng.standard_normal(m[p])))
        return out
    b = draw(x)
    it, t0 = 0, time.perf_counter()
    while True:
        taus = np.stack([O.tau_full(b[p], gw[p]) for p in range(P)])
        if kind == "curn_red":
            rr, _ = O.rho_grid_cdf_red(taus, 10 ** (2 * x[rind]), rng.random((P, 30)), 1e-20, 1e-8)
            x[hind] = 0.5 * np.log10(rr.ravel())
        irn = (np.stack([10 ** (2 * x[hind[p * 30:(p + 1) * 30]]) for p in range(P)])
               if kind == "curn_red" else np.zeros_like(taus))
        rr, _ = O.rho_grid_cdf_curn(taus, irn, rng.random(30), 1e-18, 1e-8)
        x[rind] = 0.5 * np.log10(rr)
        b = draw(x)
        it += 1
        el = time.perf_counter() - t0
        if el > seconds:
            break
    return dict(value=it / el, unit="iters/s", cores=1, kind="port",
                sample=f"{it} sweeps of the 45-pulsar {kind} loop (oracle restatement of "
                       f"pta_gibbs.py:664-704, numpy SVD, 1 thread) in {el:.1f} s")


def bench_pta(kind, C, K, W, rank, world, dev, ctx, curn_mode="exact", graph=True, shard="chain"):
    """Configs 3/4: PTAChains over the 45 simulated pulsars.  shard='chain': C chains per
    GPU, no collective (weak).  shard='pulsar' (N > 1): every rank runs the same C chains
    over its pulsar block (balanced by m^3) and exchanges per sweep over RCCL -- the
    tau-sum all-reduce for CURN (sufficient statistic) or the [tau | x_red] all-gather for
    CURN + red (strong scaling over pulsars)."""
    from pulsar_timing_gibbsspec_amd import synthetic
    from pulsar_timing_gibbsspec_amd.distributed import PulsarAllGather, TauSumAllReduce
    from pulsar_timing_gibbsspec_amd.engine import DeviceModel, PTAChains
    pta = synthetic.array_pta(kind=kind, seed=0)
    T, N, R = pta.get_basis(), pta.get_ndiag({}), pta.get_residuals()
    names = pta.param_names
    rind = [i for i, n in enumerate(names) if "rho" in n and "gw" in n]
    hind = np.array([i for i, n in enumerate(names) if "red" in n and "rho" in n])
    gwid = [np.arange(t.shape[1] - 60, t.shape[1]) for t in T]
    fixed = [np.full(t.shape[1] - 60, 1e-40) for t in T]
    red_col = hind.reshape(len(T), -1) if kind == "curn_red" else None
    sharded = shard == "pulsar" and world > 1
    if sharded:
        lo, hi = _contiguous_balanced(np.array([t.shape[1] ** 3 for t in T], float), rank, world)
        model = DeviceModel(ctx, T[lo:hi], N[lo:hi], R[lo:hi], gwid[lo:hi], fixed[lo:hi])
        x0 = np.random.default_rng(0).uniform(-9, -4, (C, len(names)))
        bounds = [_contiguous_balanced(np.array([t.shape[1] ** 3 for t in T], float), r, world)
                  for r in range(world)]
        assign = [np.arange(a, b) for a, b in bounds]
        ex = dict(allreduce=TauSumAllReduce()) if curn_mode == "sum" else \
            dict(gather=PulsarAllGather(assign, ((2 if red_col is not None else 1), 30, C), device=dev))
        eng = PTAChains(model, len(names), rind, red_col, (1e-18, 1e-8), (1e-20, 1e-8), C, x0,
                        P_global=len(T), psr_lo=lo, curn_mode=curn_mode, **ex)
        graph = False
    else:
        model = DeviceModel(ctx, T, N, R, gwid, fixed)
        x0 = np.random.default_rng(rank).uniform(-9, -4, (C, len(names)))
        eng = PTAChains(model, len(names), rind, red_col, (1e-18, 1e-8), (1e-20, 1e-8), C, x0,
                        chain_base=rank * C, curn_mode=curn_mode)
    rec = torch.empty(K, C, len(names), dtype=torch.float64, device=dev)
    for _ in range(max(1, W)):
        eng.sweep(x_rec=rec[0])
    if graph:                              # the K timed sweeps as one hipGraph replay
        eng.capture(K)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    if graph:
        eng.replay()
    else:
        for i in range(K):
            eng.sweep(x_rec=rec[i])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    if eng.info.cpu().numpy().any():
        raise RuntimeError("non-PD Sigma in the PTA bench")
    total_chains = C if sharded else C * world
    return dict(value=total_chains * K / el, unit="chain-iters/s", ms_per_step=el / K * 1e3, steps=K,
                chains_per_gpu=C, n_psr=len(T), n_param=len(names), hipgraph=bool(graph),
                sharding=("pulsars over %d GPUs (RCCL %s per sweep), strong" %
                          (world, "all-reduce" if curn_mode == "sum" else "all-gather")) if sharded
                else "chains, weak")


def _contiguous_balanced(w, rank, world):
    """Contiguous pulsar block of this rank with ~equal sum of weights (m^3 ~ b|rho cost)."""
    cw = np.concatenate([[0.0], np.cumsum(w)])
    cuts = [int(np.searchsorted(cw, cw[-1] * r / world)) for r in range(world + 1)]
    cuts[0], cuts[-1] = 0, len(w)
    for r in range(1, world):                     # every rank keeps at least one pulsar
        cuts[r] = min(max(cuts[r], cuts[r - 1] + 1), len(w) - (world - r))
    return cuts[rank], cuts[rank + 1]


def config5_cpu_baseline(seconds=10.0):
    """The oracle's restatement of one PulsarBlockGibbs sweep with white noise
    (pulsar_gibbs.py:656-698: TNT, SVD draw, aclength=20 white MH steps each recomputing
    r - T b and the white likelihood as :523-546 does, analytic rho) on ONE pulsar of the
    config-5 array (10^4 TOAs, m = 216), 1 thread; reported as array sweeps/s = 1 /
    (200 x the per-pulsar sweep time)."""
    from oracle import gibbs_oracle as O
    from pulsar_timing_gibbsspec_amd import synthetic
    d = synthetic.config5_array(n_psr=1, seed=1)
    T, r, sig, bk = d["T"][0], d["r"][0], d["sigma"][0], d["backend"][0]
    rng = np.random.default_rng(0)
    x = d["x0"][0].copy()
    gw = d["gw_cols"]
    wind = [w[0] for w in d["white"]]
    nb = len(wind) // 2
    lo = np.array([w[3] for w in d["white"]])
    hi = np.array([w[4] for w in d["white"]])
    m = T.shape[1]
    n_tm = m - 2 * gw.size

    def N_of(xx):
        return O.ndiag_white(sig, bk, xx[[2 * k for k in range(nb)]], xx[[2 * k + 1 for k in range(nb)]])
    b = np.zeros(m)
    it, t0 = 0, time.perf_counter()
    while True:
        N = N_of(x)
        TNT, dd = O.tnt(T, N, r)
        ph = np.full(m, 1e-40)
        ph[:gw.size * 2] = 1 / np.repeat(10 ** (2 * x[gw]), 2)
        b = O.bdraw_svd(TNT, dd, ph, rng.standard_normal(m))
        ll0 = O.lnlike_white(r, T, b, N_of(x))
        for _ in range(20):
            q = x.copy()
            j = rng.integers(len(wind))
            q[wind[j]] += rng.standard_normal() * 0.05 * len(wind) * rng.choice([0.1, 0.5, 1, 3, 10])
            if lo[j] <= q[wind[j]] <= hi[j]:
                ll1 = O.lnlike_white(r, T, b, N_of(q))
                if ll1 - ll0 > np.log(rng.random()):
                    x, ll0 = q, ll1
        tau = O.tau_half(b, np.arange(2 * gw.size))
        x[gw] = 0.5 * np.log10(O.rho_analytic(tau, rng.random(gw.size), d["rhomin"], d["rhomax"]))
        it += 1
        el = time.perf_counter() - t0
        if el > seconds:
            break
    per_psr = el / it
    return dict(value=1.0 / (200 * per_psr), unit="iters/s", cores=1, kind="port",
                sample=f"{it} single-pulsar sweeps (10^4 TOAs, m={m}, n_tm={n_tm}, 20 white MH steps) of the "
                       f"oracle restatement of pulsar_gibbs.py:656-698 + :373-404 in {el:.1f} s, "
                       f"{per_psr * 1e3:.0f} ms/pulsar, scaled to the 200-pulsar array")


def bench_config5(C, K, W, rank, world, dev, n_psr=200, n_toa=10_000, n_f=100, aclength=20, reps=5):
    """BASELINE configs[4]: n_psr independent pulsars x C chains per GPU, white-noise MH
    (aclength steps) forcing the per-chain TNT (batched SYRK) every sweep."""
    from pulsar_timing_gibbsspec_amd import _lib, synthetic
    from pulsar_timing_gibbsspec_amd.white import WhiteArrayChains, WhiteNoiseModel
    d = synthetic.config5_array(n_psr=n_psr, n_toa=n_toa, n_f=n_f, seed=0)
    ctx = _lib.Context(dev.index, seed=20251016)
    ctx.set_option(_lib.OPT_X_PER_SYS, 1)
    wm = WhiteNoiseModel(ctx, d["T"], d["r"], d["sigma"], d["backend"], [d["fidx"]] * n_psr,
                         [d["phiinv_fixed"]] * n_psr, [d["white"]] * n_psr, C)
    m = int(wm.m[0])
    del d["T"]
    eng = WhiteArrayChains(wm, d["n_param"], d["gw_cols"], d["rhomin"], d["rhomax"],
                           np.repeat(d["x0"], C, axis=0), aclength=aclength, chain_base=rank * C)
    for _ in range(W):
        eng.sweep()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(K):
        eng.sweep()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    if eng.info.cpu().numpy().any() or int(wm.pinfo.abs().sum()):
        raise RuntimeError("non-PD system in the config-5 bench")
    # the dominant kernel: gs_white_tnt (k_white_syrk), timed alone on the ctx stream
    stream = ctx.stream
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(reps):
        wm.refresh(eng.x, eng.n_param)
    e1.record(stream)
    torch.cuda.synchronize()
    refresh_ms = e0.elapsed_time(e1) / reps
    n_sys = n_psr * C
    flops = n_sys * (n_toa * m * (m + 1) + 2 * n_toa * m)      # SYRK + TNr per system
    tflops = flops / (refresh_ms * 1e-3) / 1e12
    return dict(value=C * world * K / el, unit="chain-iters/s", ms_per_step=el / K * 1e3, steps=K,
                chains_per_gpu=C, n_psr=n_psr, n_toa=n_toa, m=m, aclength=aclength,
                roofline={"bound": "mfma", "kernel": "k_white_syrk + k_prefix (gs_white_tnt + gs_prefix_sys)",
                          "achieved": tflops, "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                          "frac": tflops / FP64_PEAK_TFLOPS, "kernel_avg_ms": refresh_ms,
                          "alg_flops_per_launch": flops,
                          "note": "per-chain TNT/d of all 200 pulsars (n m (m+1) + 2 n m flop per system) "
                                  "over the HIP-event time of one refresh (SYRK + prefix)"})


def ecorr_white_cpu_baseline(seconds=10.0, aclength=10):
    """The oracle's restatement of the white + ECORR sweep (notebook order: white MH on
    get_lnlikelihood_white :523-546, TNT recomputed with the new N as the reference's reset
    forces, ECORR MH on get_lnlikelihood_fullmarg, rho|b, SVD b draw), one chain, 1 thread."""
    from oracle import gibbs_oracle as O
    from pulsar_timing_gibbsspec_amd import synthetic
    pta = synthetic.ecorr_pulsar_pta("J1713+0747", seed=0, white_vary=True)
    T, r = pta.get_basis()[0], pta.get_residuals()[0]
    names = pta.param_names
    wn = pta.models[0].white[0]
    ebk = pta.signals["J1713+0747_basis_ecorr"].epoch_backend
    eind = [i for i, n in enumerate(names) if "ecorr" in n]
    ef_i = [i for i, n in enumerate(names) if n.endswith("efac")]
    eq_i = [i for i, n in enumerate(names) if "equad" in n]
    wind = sorted(ef_i + eq_i)
    gw = np.array([i for i, n in enumerate(names) if "rho" in n])
    m, ne = T.shape[1], ebk.size
    gwid = ne + np.arange(2 * gw.size)
    lo = np.array([0.1 if i in ef_i else -8.5 for i in range(len(names))])
    hi = np.array([5.0 if i in ef_i else -5.0 for i in range(len(names))])
    rng = np.random.default_rng(0)
    x = np.zeros(len(names))
    x[ef_i], x[eq_i], x[eind] = 1.0, -7.0, -6.3
    x[gw] = rng.uniform(-9, -4, gw.size)

    def N_of(xx):
        return O.ndiag_white(wn.sigma, wn.backends, xx[ef_i], xx[eq_i])

    def phi(xx):
        ph = np.full(m, 1e40)
        ph[:ne] = (10.0 ** (2.0 * xx[eind]))[ebk]
        ph[gwid] = np.repeat(10.0 ** (2.0 * xx[gw]), 2)
        return ph

    def prior(ind):
        return lambda xx: 0.0 if np.all((xx[ind] >= lo[ind]) & (xx[ind] <= hi[ind])) else -np.inf

    def steps(ind):
        return [(rng.choice([0.1, 0.5, 1, 3, 10], p=[.1, .15, .5, .15, .1]), rng.choice(ind),
                 rng.standard_normal(), rng.random()) for _ in range(aclength)]
    TNT, dd = O.tnt(T, N_of(x), r)
    b = O.bdraw_svd(TNT, dd, 1.0 / phi(x), rng.standard_normal(m))
    it, t0 = 0, time.perf_counter()
    while True:
        x = O.white_mh(x, wind, steps(wind), lambda xx: O.lnlike_white(r, T, b, N_of(xx)), prior(wind))
        N = N_of(x)
        TNT, dd = O.tnt(T, N, r)

        def lnl(xx):
            ph = phi(xx)
            return O.lnlike_fullmarg(r, N, TNT, dd, 1.0 / ph, np.sum(np.log(ph)))
        x = O.white_mh(x, eind, steps(eind), lnl, prior(eind))
        x[gw] = 0.5 * np.log10(O.rho_analytic(O.tau_half(b, gwid), rng.random(gw.size), 1e-18, 1e-8))
        b = O.bdraw_svd(TNT, dd, 1.0 / phi(x), rng.standard_normal(m))
        it += 1
        el = time.perf_counter() - t0
        if el > seconds:
            break
    return dict(value=it / el, unit="iters/s", cores=1, kind="port",
                sample=f"{it} sweeps of the single-chain white + ECORR loop (m={m}, {ne} epochs, {aclength} white + "
                       f"{aclength} ECORR MH steps, oracle restatement, numpy/LAPACK, 1 thread) in {el:.1f} s")


def ecorr_cpu_baseline(seconds=10.0, aclength=10):
    """The oracle's restatement of the ECORR sweep (notebook order; update_ecorr_params
    :456-484 on get_lnlikelihood_fullmarg :569-610 with TNT recomputed each sweep as the
    reference does, :664-665; SVD b draw :489-520), one chain, 1 thread."""
    from oracle import gibbs_oracle as O
    from pulsar_timing_gibbsspec_amd import synthetic
    pta = synthetic.ecorr_pulsar_pta("J1713+0747", seed=0)
    T, r, N = pta.get_basis()[0], pta.get_residuals()[0], pta.get_ndiag()[0]
    names = pta.param_names
    sig = pta.signals["J1713+0747_basis_ecorr"]
    ebk = sig.epoch_backend
    eind = [i for i, n in enumerate(names) if "ecorr" in n]
    gw = np.array([i for i, n in enumerate(names) if "rho" in n])
    m = T.shape[1]
    ne = ebk.size
    gwid = ne + np.arange(2 * gw.size)
    rng = np.random.default_rng(0)
    x = np.concatenate([[-6.3] * len(eind), rng.uniform(-9, -4, gw.size)])

    def phi(xx):
        ph = np.full(m, 1e40)
        ph[:ne] = (10.0 ** (2.0 * xx[eind]))[ebk]
        ph[gwid] = np.repeat(10.0 ** (2.0 * xx[gw]), 2)
        return ph
    TNT, dd = O.tnt(T, N, r)
    b = O.bdraw_svd(TNT, dd, 1.0 / phi(x), rng.standard_normal(m))    # first b from xs
    it, t0 = 0, time.perf_counter()
    while True:
        TNT, dd = O.tnt(T, N, r)

        def lnl(xx):
            ph = phi(xx)
            return O.lnlike_fullmarg(r, N, TNT, dd, 1.0 / ph, np.sum(np.log(ph)))
        steps = [(rng.choice([0.1, 0.5, 1, 3, 10], p=[.1, .15, .5, .15, .1]), rng.choice(eind),
                  rng.standard_normal(), rng.random()) for _ in range(aclength)]
        x = O.white_mh(x, eind, steps, lnl, lambda xx: 0.0 if np.all((xx[eind] >= -8.5) & (xx[eind] <= -5)) else -np.inf)
        x[gw] = 0.5 * np.log10(O.rho_analytic(O.tau_half(b, gwid), rng.random(gw.size), 1e-18, 1e-8))
        b = O.bdraw_svd(TNT, dd, 1.0 / phi(x), rng.standard_normal(m))
        it += 1
        el = time.perf_counter() - t0
        if el > seconds:
            break
    return dict(value=it / el, unit="iters/s", cores=1, kind="port",
                sample=f"{it} sweeps of the single-chain ECORR loop (m={m}, {ne} epochs, {aclength} ECORR MH steps, "
                       f"oracle restatement, numpy/LAPACK, 1 thread) in {el:.1f} s")


def _ecorr_traffic(C, fname="pmc_traffic_ecorr.json"):
    """HBM bytes per launch of k_ecorr_prefix<likelihood> from the committed PMC passes
    (tools/gpu_pmc_ecorr.sh -> profiles/pmc_traffic_ecorr.json for the shared-operand kernel,
    profiles/pmc_traffic_ecorr_white.json for the per-chain-operand one), same chain count only."""
    try:
        d = json.load(open(os.path.join(ROOT, "profiles", fname)))
    except (OSError, ValueError):
        return None
    return d.get("bytes_per_launch") if d.get("chains") == C else None


def bench_ecorr_white(C, K, W, rank, world, dev, aclength=10):
    """SURVEY 8f-4 with white noise sampled too (the notebook's J1713 configuration): per sweep
    white MH (aclength steps) -> per-chain TNT (gs_white_tnt) -> per-chain ECORR operands ->
    ECORR MH (aclength steps) -> rho|b -> gated b, C chains per GPU."""
    from pulsar_timing_gibbsspec_amd import _lib, synthetic
    from pulsar_timing_gibbsspec_amd.ecorr import EcorrWhiteChains, white_ecorr_models
    pta = synthetic.ecorr_pulsar_pta("J1713+0747", seed=0, white_vary=True)
    names = pta.param_names
    sig = pta.signals["J1713+0747_basis_ecorr"]
    wn = pta.models[0].white[0]
    ebk = sig.epoch_backend
    ne = ebk.size
    eind = [i for i, n in enumerate(names) if "ecorr" in n]
    wind = [i for i, n in enumerate(names) if "efac" in n or "equad" in n]
    gw = [i for i, n in enumerate(names) if "rho" in n]
    T = pta.get_basis()[0]
    m = T.shape[1]
    gwid = ne + np.arange(2 * len(gw))
    wl = [(j, 0 if names[j].endswith("efac") else 1, int(names[j].split("_b")[1].split("_")[0]),
           0.1 if names[j].endswith("efac") else -8.5, 5.0 if names[j].endswith("efac") else -5.0) for j in wind]
    ctx = _lib.Context(dev.index, seed=20251018)
    wm, wmR, em = white_ecorr_models(ctx, T, pta.get_residuals()[0], wn.sigma, wn.backends, gwid, wl, np.arange(ne),
                                     ebk, eind, [-8.5] * len(eind), [-5.0] * len(eind), len(names), C)
    rng = np.random.default_rng(100 + rank)
    x0 = np.empty((C, len(names)))
    x0[:, wind] = [1.0 if names[j].endswith("efac") else -7.0 for j in wind]
    x0[:, eind] = -6.3
    x0[:, gw] = rng.uniform(-9, -4, (C, len(gw)))
    eng = EcorrWhiteChains(wm, em, gw, gwid, 1e-18, 1e-8, x0, aclength, aclength, chain_base=rank * C, wmR=wmR)
    for _ in range(W):
        eng.sweep()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(K):
        eng.sweep()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    if int(em.binfo.abs().sum()) or int(em.pinfo.abs().sum()):
        raise RuntimeError("non-PD system in the white + ECORR bench")
    # dominant kernel: gs_ecorr_prefix in likelihood mode on per-chain operands, timed alone
    stream = ctx.stream
    eng._phiinv(False)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 10
    e0.record(stream)
    for _ in range(reps):
        em._eval(eng.x, eng.phiinv_F)
    e1.record(stream)
    torch.cuda.synchronize()
    k_ms = e0.elapsed_time(e1) / reps
    mR, NF, nM = em.mR, em.NF, em.nm
    flops = C * (ne * (mR + 1) * (mR + 2) + nM * (NF + 1) * (NF + 2) + (NF + 1) ** 3 // 3)
    tflops = flops / (k_ms * 1e-3) / 1e12
    return dict(value=C * world * K / el, unit="chain-iters/s", ms_per_step=el / K * 1e3, steps=K,
                chains_per_gpu=C, m=m, n_epoch=ne, aclength_white=aclength, aclength_ecorr=aclength,
                roofline={"bound": "mfma", "kernel": "k_ecorr_prefix<likelihood mode, per-chain operands>",
                          "achieved": tflops, "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                          "frac": tflops / FP64_PEAK_TFLOPS, "kernel_avg_ms": k_ms, "alg_flops_per_launch": flops,
                          "traffic": _ecorr_traffic(C, "pmc_traffic_ecorr_white.json"),
                          "note": "as the ecorr line; each chain's [B | d_E] rows stream from HBM (343 MB of "
                                  "algorithmic reads per 4096-chain launch; traffic = PMC FETCH_SIZE x2 + "
                                  "WRITE_SIZE, the x2 wide-read correction makes it an upper estimate)"},
                config="SURVEY 8f-4 with EFAC/EQUAD sampled: J1713-like pulsar, 2 backends, 136 ECORR epochs, "
                       "white MH + per-chain TNT + ECORR MH + analytic rho|b + gated b per sweep, chain-sharded")


def bench_ecorr(C, K, W, rank, world, dev, aclength=10, reps=10):
    """single pulsar with basis ECORR (J1713-like, 2 backends, 136 epochs,
    m = 212), C chains per GPU, aclength ECORR MH steps per sweep (each a batched
    likelihood evaluation: k_ecorr_schur + prefix + lnlike), analytic rho|b, gated b."""
    from pulsar_timing_gibbsspec_amd import _lib, synthetic
    from pulsar_timing_gibbsspec_amd.ecorr import EcorrFreeSpectrumChains, EcorrModel
    pta = synthetic.ecorr_pulsar_pta("J1713+0747", seed=0)
    names = pta.param_names
    sig = pta.signals["J1713+0747_basis_ecorr"]
    ebk = sig.epoch_backend
    ne = ebk.size
    eind = [i for i, n in enumerate(names) if "ecorr" in n]
    gw = [i for i, n in enumerate(names) if "rho" in n]
    T = pta.get_basis()[0]
    m = T.shape[1]
    gwid = ne + np.arange(2 * len(gw))
    ctx = _lib.Context(dev.index, seed=20251017)
    em = EcorrModel(ctx, T, pta.get_ndiag()[0], pta.get_residuals()[0], np.arange(ne), ebk, gwid, eind,
                    [-8.5] * len(eind), [-5.0] * len(eind), len(names), C)
    rng = np.random.default_rng(rank)
    x0 = np.concatenate([np.full((C, len(eind)), -6.3), rng.uniform(-9, -4, (C, len(gw)))], axis=1)
    eng = EcorrFreeSpectrumChains(em, gw, gwid, 1e-18, 1e-8, x0, aclength=aclength, chain_base=rank * C)
    for _ in range(W):
        eng.sweep()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(K):
        eng.sweep()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    if int(em.binfo.abs().sum()) or int(em.pinfo.abs().sum()):
        raise RuntimeError("non-PD system in the ECORR bench")
    # dominant kernel: gs_ecorr_prefix in likelihood mode (one launch per Metropolis step:
    # epoch Schur complement + fixed-prior prefix + F-block factorisation), timed alone
    stream = ctx.stream
    em.factor(eng.x)
    eng._phiinv(False)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(reps):
        em._eval(eng.x, eng.phiinv_F)
    e1.record(stream)
    torch.cuda.synchronize()
    k_ms = e0.elapsed_time(e1) / reps
    mR, NF, nM = em.mR, em.NF, em.nm
    # epoch-weighted SYRK (lower triangle of [B | d_E]^T W [B | d_E]) + the fixed-prior Schur
    # update + the (NF+1)-augmented Cholesky of the free-spectrum block
    flops = C * (ne * (mR + 1) * (mR + 2) + nM * (NF + 1) * (NF + 2) + (NF + 1) ** 3 // 3)
    tflops = flops / (k_ms * 1e-3) / 1e12
    return dict(value=C * world * K / el, unit="chain-iters/s", ms_per_step=el / K * 1e3, steps=K,
                chains_per_gpu=C, m=m, n_epoch=ne, m_R=mR, aclength=aclength,
                roofline={"bound": "mfma", "kernel": ("k_ecorr_prefix<likelihood mode>" if em.fused and em.fused_lnl
                                                      else "k_ecorr_schur + k_prefix + k_lnlike_marg"),
                          "achieved": tflops,
                          "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s", "frac": tflops / FP64_PEAK_TFLOPS,
                          "kernel_avg_ms": k_ms, "alg_flops_per_launch": flops,
                          "traffic": _ecorr_traffic(C),
                          "note": "ne (mR+1)(mR+2) + nM (NF+1)(NF+2) + (NF+1)^3/3 flop per chain (epoch-weighted "
                                  "SYRK with the d_E row + fixed-prior Schur update + F-block Cholesky) over the "
                                  "HIP-event time of one all-chain likelihood launch"},
                config="SURVEY 8f-4: J1713-like pulsar, basis ECORR (2 backends, 136 epochs) + 30-bin free "
                       "spectrum + 16-col TM, ECORR MH + analytic rho|b + gated b per sweep, chain-sharded")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=500)
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--chains", type=int, default=4096, help="chains per GPU")
    ap.add_argument("--sweeps-per-launch", type=int, default=100)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--bcast", type=int, default=None, help="GS_OPT_BCAST (0 readlane, 1 LDS, 2 batched)")
    ap.add_argument("--pta", default="curn_red,curn", help="secondary PTA configs measured in the same run "
                    "(comma list of curn_red, curn; or none). curn uses the sufficient-statistic draw")
    ap.add_argument("--pta-chains", type=int, default=2048,
                    help="chains per GPU for the PTA lines (measured: 256 -> 1024 -> 2048 -> 4096 chains give "
                         "CURN + red 3.0e5 -> 3.8e5 -> 3.9e5 -> 4.0e5 chain-it/s: saturated at 2048)")
    ap.add_argument("--pta-steps", type=int, default=20)
    ap.add_argument("--config5", type=int, default=1, help="measure BASELINE configs[4] too (1/0)")
    ap.add_argument("--pta-graph", type=int, default=0, help="time the PTA sweeps as a hipGraph replay (1/0); "
                    "measured no faster: the sweeps are GPU-bound and eager launches queue ahead")
    ap.add_argument("--pta-shard", default="chain", help="chain | pulsar: how N > 1 GPUs split the PTA configs")
    ap.add_argument("--ecorr", type=int, default=1, help="measure the basis-ECORR path (SURVEY 8f-4) too (1/0)")
    ap.add_argument("--ecorr-chains", type=int, default=4096)
    ap.add_argument("--ecorr-steps", type=int, default=10)
    ap.add_argument("--c5-chains", type=int, default=16)
    ap.add_argument("--c5-steps", type=int, default=5)
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # one process per GPU over RCCL; GS_DIST_BACKEND=gloo (and more ranks than GPUs, ranks
    # sharing devices round-robin) only to rehearse the multi-rank paths on one GPU
    backend = os.environ.get("GS_DIST_BACKEND", "nccl")
    if backend != "nccl":
        local = local % torch.cuda.device_count()
    if world > 1:
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    from pulsar_timing_gibbsspec_amd import _lib, synthetic
    from pulsar_timing_gibbsspec_amd.engine import DeviceModel, FreeSpectrumChains

    pta = synthetic.single_pulsar_pta("J1713+0747", seed=0)
    T, N, r = pta.get_basis()[0], pta.get_ndiag({})[0], pta.get_residuals()[0]
    gwid = np.arange(60)
    ctx = _lib.Context(local, seed=20251015)
    if args.bcast is not None:
        ctx.set_option(_lib.OPT_BCAST, args.bcast)
    model = DeviceModel(ctx, [T], [N], [r], [gwid], [np.full(T.shape[1] - 60, 1e-40)])
    C = args.chains
    x0 = np.random.default_rng(rank).uniform(-9, -4, (C, 30))
    run = FreeSpectrumChains(model, 1e-18, 1e-8, C, x0, chain_base=rank * C)
    K, W, S = args.steps, args.warmup, max(1, args.sweeps_per_launch)
    m = int(model.m[0])
    x_rec = torch.empty(K, C, 30, dtype=torch.float64, device=dev)
    b_rec = torch.empty(K, C, model.ldb, dtype=torch.float64, device=dev)

    # warmup (untimed)
    done = 0
    while done < W:
        n = min(S, W - done)
        run.run(n, x_rec=x_rec[:n], b_rec=b_rec[:n])
        done += n
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    stream = ctx.stream
    evs = []
    t0 = time.perf_counter()
    done = 0
    while done < K:
        n = min(S, K - done)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        run.run(n, x_rec=x_rec[done:done + n], b_rec=b_rec[done:done + n])
        e1.record(stream)
        evs.append((e0, e1, n))
        done += n
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    info = run.info.cpu().numpy()
    if info.any():
        raise RuntimeError(f"{int((info != 0).sum())} chains hit a non-PD Sigma")

    total_chains = C * world
    value = total_chains * K / el
    # roofline of the fused sweep kernel (dominant kernel: one launch per S sweeps)
    kern_ms = np.array([a.elapsed_time(b) for a, b, _ in evs])
    sweeps = np.array([n for _, _, n in evs])
    per_sweep_s = float(np.sum(kern_ms) / 1e3 / np.sum(sweeps))
    alg_flops_launch = flops_per_chain_sweep(m) * C * S
    launch_s = per_sweep_s * S
    achieved = alg_flops_launch / launch_s / 1e12
    exe = executed_flops_per_chain_sweep(model.NF, int(model.nm[0])) * C * S / launch_s / 1e12
    xh = x_rec.cpu().numpy()
    ess = ess_min_bin(xh, el, total_chains)

    out = None
    if rank == 0:
        out = {
            "metric": "Gibbs iters/sec (all chains, whole node) + ESS/sec of log10_rho",
            "value": value, "unit": "chain-iters/s", "n_gpus": world, "steps": K, "warmup": W,
            "ms_per_step": el / K * 1e3, "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "f64", "data": "synthetic",
            "config": {"workload": "configs[1]: J1713+0747 sim (720 TOAs, m=76, 30-bin free spectrum), "
                                   f"{C} independent chains per GPU", "chains_per_gpu": C,
                       "global_chains": total_chains, "m": m, "n_f": 30,
                       "sweeps_per_launch": S, "bcast": ctx.get_option(_lib.OPT_BCAST),
                       "parallelism": f"chains sharded over {world} GPU(s)"},
            "ess_per_s": ess,
            "roofline": {"bound": "mfma", "achieved": achieved, "peak": FP64_PEAK_TFLOPS,
                         "unit": "TFLOP/s", "frac": achieved / FP64_PEAK_TFLOPS,
                         "traffic": pmc_traffic(S, C),
                         "kernel": "k_sweep_freespec", "kernel_avg_ms": launch_s * 1e3,
                         "alg_flops_per_launch": alg_flops_launch,
                         "executed_tflops": exe, "executed_frac": exe / FP64_PEAK_TFLOPS},
        }
        if not args.no_cpu_baseline and world == 1:  # rank 0 at N=1 only
            out["cpu_baseline"] = cpu_baseline(args.cpu_seconds)
    for kind in [k for k in args.pta.split(",") if k and k != "none"]:
        mode = "sum" if kind == "curn" else "exact"
        sec = bench_pta(kind, args.pta_chains, args.pta_steps, 2, rank, world, dev, ctx, curn_mode=mode,
                        graph=bool(args.pta_graph), shard=args.pta_shard)
        if rank == 0:
            sec["config"] = (f"configs[3]: 45-pulsar CURN{' + per-pulsar red' if kind == 'curn_red' else ''} "
                             f"free spectrum, chain-sharded, common draw {mode}")
            if not args.no_cpu_baseline and world == 1:
                sec["cpu_baseline"] = pta_cpu_baseline(kind, args.cpu_seconds)
            out.setdefault("secondary", {})[kind] = sec
    if args.ecorr:
        sec = bench_ecorr(args.ecorr_chains, args.ecorr_steps, 2, rank, world, dev)
        if rank == 0:
            sec["sharding"] = "chains, weak"
            if not args.no_cpu_baseline and world == 1:
                sec["cpu_baseline"] = ecorr_cpu_baseline(args.cpu_seconds)
            out.setdefault("secondary", {})["ecorr"] = sec
        sec = bench_ecorr_white(args.ecorr_chains, args.ecorr_steps, 2, rank, world, dev)
        if rank == 0:
            sec["sharding"] = "chains, weak"
            if not args.no_cpu_baseline and world == 1:
                sec["cpu_baseline"] = ecorr_white_cpu_baseline(args.cpu_seconds)
            out["secondary"]["ecorr_white"] = sec
    if args.config5:
        sec = bench_config5(args.c5_chains, args.c5_steps, 1, rank, world, dev)
        if rank == 0:
            sec["config"] = ("configs[4]: 200 synthetic pulsars x 10^4 TOAs x 100 frequencies (m=216), "
                             "white-noise MH (20 steps) + per-chain TNT recompute every sweep, chain-sharded")
            if not args.no_cpu_baseline and world == 1:
                sec["cpu_baseline"] = config5_cpu_baseline(args.cpu_seconds)
            out.setdefault("secondary", {})["config5"] = sec
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
