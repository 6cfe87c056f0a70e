"""Benchmark: Gibbs iterations/s (all chains, whole node) + ESS/s of log10 rho.

Workload (BASELINE.json configs[1]): the simulated J1713+0747 pulsar (720 TOAs,
30-bin free spectrum + 16-column timing model, m = 76, fixed white noise),
``--chains`` independent chains per GPU (default 4096), batched on each MI355X.
A "step" = one fused launch of ``--sweeps-per-launch`` (100) Gibbs sweeps of every
chain (rho|b then b|rho, each sweep's chain rows recorded to HBM as
PulsarBlockGibbs.sample records them; 100 = the reference's save cadence,
pulsar_gibbs.py:701-710).  ``value`` counts chain-sweeps: chains x steps x 100 / time.
ESS/s = value x (ESS per chain-sweep of the worst bin), the ESS fraction from a
separate untimed 2000-sweep run (``--ess-sweeps``).

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
    """HBM bytes per launch of the headline's fused-sweep kernel from the committed PMC profile
    (profiles/pmc_traffic.json: FETCH_SIZE / WRITE_SIZE passes, tools/gpu_r06m.sh), valid for the same
    launch shape."""
    f = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        d = json.load(open(f))
    except (OSError, ValueError):
        return None
    if d.get("sweeps_per_launch") != S or d.get("chains") != C or "bytes_per_launch" not in d:
        return None
    return d["bytes_per_launch"]


def gpu_ess(block, kind):
    """The GPU leg of the ESS comparison.  ``block(n_max, rec)`` advances the engine by n <= n_max
    sweeps and returns (n, rows): rows = the (n, chains, k) device tensor of the recorded log10 rho
    columns when ``rec``, else None.  The run lengths (burn-in, recorded sweeps) are the CPU leg's
    (diagnostics.ESS_RUN) and so is the estimator (diagnostics.ess_summary: pooled ACF over the
    chains, Sokal window, standard error from Sokal's variance): the two legs' ESS per sweep compare
    like for like."""
    from pulsar_timing_gibbsspec_amd.diagnostics import ESS_RUN, ess_summary
    burn, sweeps = ESS_RUN[kind]
    done = 0
    while done < burn:
        done += block(burn - done, False)[0]
    parts, done = [], 0
    while done < sweeps:
        n, rows = block(sweeps - done, True)
        parts.append(rows.to("cpu", copy=True))
        done += n
    X = torch.cat(parts).permute(1, 0, 2).contiguous().numpy()      # (chains, sweeps, k)
    return ess_summary(X, burn)


def sweep_block(eng, cols, chains=None):
    """gpu_ess's block for an engine with .sweep() and .x (chains, n_param): one sweep per call,
    the x columns ``cols`` of the first ``chains`` chains recorded."""
    idx = torch.as_tensor(np.asarray(cols), dtype=torch.long, device=eng.x.device)
    ce = chains or eng.x.shape[0]

    def block(n_max, rec):
        eng.sweep()
        return 1, (eng.x[:ce].index_select(1, idx).unsqueeze(0) if rec else None)
    return block


def timed_region(world, dev, fn):
    """barrier + synchronize, fn(), synchronize + barrier; wall seconds, max over ranks."""
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    fn()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    return el


# untimed warm-up of every secondary line: the line's own sweeps for at least this long (and at least
# the line's W), since the shader clock ramps back up over ~10-20 ms of sustained load after the idle
# host-side setup between lines (profiles/r05z2/launch_stats.log: the first launches of each kernel
# 10-15 % slower).  The headline keeps exactly the driver's --warmup steps.
WARM_MS = 60.0


def warm(fn, min_calls=1, min_ms=WARM_MS):
    """Call fn() (one untimed sweep / launch of the line) at least min_calls times and until min_ms of
    wall time has passed, synchronising every few calls so the wall time follows the GPU.  With more
    than one rank every rank makes the SAME number of calls (fn may hold a collective: the pulsar-sharded
    lines' per-sweep exchange): min_calls first, then the extra calls the slowest rank needs to reach
    min_ms, agreed by an all-reduce while no rank is inside fn."""
    t0 = time.perf_counter()
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        for _ in range(min_calls):
            fn()
        torch.cuda.synchronize()
        el = (time.perf_counter() - t0) * 1e3
        per = el / max(1, min_calls)
        extra = 0 if el >= min_ms else int(np.ceil((min_ms - el) / max(per, 1e-3)))
        dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" else "cpu"
        t = torch.tensor([extra], dtype=torch.int64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        extra = int(t.item())
        for i in range(extra):
            fn()
            if i % 4 == 3:
                torch.cuda.synchronize()
        torch.cuda.synchronize()
        return min_calls + extra
    n = 0
    while n < min_calls or (time.perf_counter() - t0) * 1e3 < min_ms:
        fn()
        n += 1
        if n % 4 == 0:
            torch.cuda.synchronize()
    torch.cuda.synchronize()
    return n


def event_ms(stream, fn, reps, warm_calls=10):
    """Average HIP-event time of fn() on ``stream`` (the context stream the C-ABI launches on),
    after at least `warm_calls` untimed calls and WARM_MS of wall time of them: the clock ramps back
    up over ~10-20 ms of sustained load after host-bound phases (rocprof r04f: the red grid kernel at
    0.84 ms right after the small ESS launches, 0.745 in the sweeps)."""
    warm(fn, warm_calls)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(reps):
        fn()
    e1.record(stream)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def grid_peak():
    """Measured ceiling of the round-2 kernels' own op mixes (tools/probe/grid_probe.hip ->
    profiles/grid_probe.json); reported beside the hardware roof as `op_mix_ceiling`."""
    try:
        return json.load(open(os.path.join(ROOT, "profiles", "grid_probe.json")))
    except (OSError, ValueError):
        return None


# Hardware VALU roof (MI355X_MICROARCH.md, 'vector-instruction ISSUE cost'; the FP64 vector peak
# 78.6 TF = 1024 SIMDs x 2.4 GHz x 16 FMA lanes per clock): a wave64 add/mul/fma/min/cmp (f64 or
# f32) issues in 4 SIMD cycles, a transcendental (v_rcp / v_exp / v_log) in 8.
SIMDS, CLOCK_HZ = 1024, 2.4e9


SWEEP_SHAPES = {1: "k_sweep_freespec (12-wave hand-off workgroups)", 2: "k_sweep_freespec (one chain per wave)",
                3: "k_sweep_pair (two chains per wave)"}


def sweep_kernel(ctx, rm=False):
    """Name of the fused-sweep kernel the context's last gs_sweep_freespec launch ran
    (GS_OPT_LAST_SWEEP_SHAPE, chosen by the library's cost model unless --sched asks)."""
    from pulsar_timing_gibbsspec_amd import _lib
    name = SWEEP_SHAPES.get(ctx.get_option(_lib.OPT_LAST_SWEEP_SHAPE), "k_sweep_freespec")
    return name.replace("k_sweep_freespec", "k_sweep_freespec_rm") if rm else name


def sq_counts():
    """Per-draw SQ instruction counts of the shipped headline kernel (one --pmc pass of SQ counters,
    tools/gpu_r06_pmc.sh -> profiles/sq_headline.json), or None."""
    try:
        d = json.load(open(os.path.join(ROOT, "profiles", "sq_headline.json")))
        return d["per_draw"]["SQ_INSTS_VALU"], d["per_draw"]["SQ_INSTS_MFMA"], d
    except (OSError, ValueError, KeyError):
        return None


def simd_issue(launch_s, draws, valu_cycles=4.5):
    """The headline kernel against the SIMD's issue capacity: on MI355X an f64 MFMA (64 cycles) does
    not overlap the SIMD's VALU (tools/probe/mfma_probe.hip, profiles/r04o/mfma_probe.txt), so a draw
    costs at least its VALU issue cycles + 64 per f64 MFMA.  Per-draw instruction counts from the
    committed SQ counters of the shipped kernel (profiles/sq_headline.json: SQ_INSTS_VALU / SQ_INSTS_MFMA
    per draw); ~4.5 SIMD cycles per VALU instruction (f64 FMA ~5, 32-bit ~2.5, profiles/valu_rate.json)."""
    sq = sq_counts()
    if sq is None:
        return None
    valu, mfma, d = sq
    cyc = launch_s * CLOCK_HZ * SIMDS / draws
    need = valu * valu_cycles + mfma * 64
    return {"simd_cycles_per_draw": cyc, "valu_per_draw": valu, "mfma_per_draw": mfma,
            "issue_cycles_per_draw": need, "frac": need / cyc, "source": "profiles/sq_headline.json",
            "sq_library_sources": d.get("library_sources"),
            "note": "fraction of the SIMD time a draw's instructions need to issue (MFMA and VALU serialise "
                    "on MI355X); the rest is dependency wait nobody fills"}


def valu_roof(plain, transc):
    """Units/s the whole chip can issue when one unit needs `plain` 4-cycle and `transc` 8-cycle
    lane operations (the grid kernels' stated minimal op counts)."""
    return SIMDS * CLOCK_HZ * 64 / (4.0 * plain + 8.0 * transc)


# minimal lane operations per unit: red grid point h e^-h (pta_gibbs.py:265-266) = gw + rho,
# 1/a, tau y, e^-h, h e^-h, the running sum and the searchsorted compare -- k_rho_red_cert16 runs
# them in f32 with two points per packed v_pk_* instruction, so its 5 plain ops cost 2.5 issue
# slots per point (4 cycles each) beside the 2 unpacked transcendentals (8 cycles each): 26
# cycles per wave-point; CURN term of the pdf product (pta_gibbs.py:192-205) = one Horner FMA
# each for the product D(rho) = prod (rho + irn) and the ratio numerator N(rho) (no per-term
# division or log; the kernel groups 4 pulsars and spends 2.5); CURN-from-sums grid point = one
# FMA (c_g - S w_g), the row max, e^x, the running sum and the compare.
GRID_MIN_OPS = {"red": (2.5, 2), "curn_term": (2, 0), "curn_sum": (4, 1)}


def cpu_line(kind, seconds):
    """cpu_baseline record: the oracle's loop, one single-thread process per host core.  A
    baseline that cannot run is reported as such rather than discarding the GPU figures."""
    from oracle.cpu_baseline import aggregate
    try:
        return aggregate(kind, seconds)
    except Exception as exc:  # noqa: BLE001
        return {"value": None, "unit": "iters/s", "kind": "port", "error": str(exc)[-500:]}


HYPER_ACL = 20     # aclength_hyper of the curn_plred line (as configs[4] fixes aclength_white = 20)


def cpu_calibration():
    """The committed reference-vs-port CPU speed ratios (tools/calibrate_cpu_baseline.py, run in
    the build container where the reference is importable), or None."""
    try:
        return json.load(open(os.path.join(ROOT, "profiles", "cpu_calibration.json")))
    except (OSError, ValueError):
        return None


def bench_pta(kind, C, K, W, rank, world, dev, ctx, shard="chain", ess=True):
    """configs[3]: PTAChains over the 45 simulated pulsars.  shard='chain': C chains per
    GPU, no collective (weak).  shard='pulsar' (N > 1): every rank runs the same C chains
    over its pulsar block (balanced by m^3) and exchanges per sweep over RCCL -- the
    tau-sum all-reduce for CURN (sufficient statistic, pta_gibbs.py:181-214) or the
    [tau | x_red] all-gather for CURN + red (strong scaling over pulsars)."""
    from pulsar_timing_gibbsspec_amd import _lib, synthetic
    from pulsar_timing_gibbsspec_amd.array_gibbs import balanced_blocks
    from pulsar_timing_gibbsspec_amd.distributed import PulsarAllGather, TauSumAllReduce
    from pulsar_timing_gibbsspec_amd.engine import DeviceModel, PTAChains
    curn_mode = "sum" if kind == "curn" else "exact"
    pta = synthetic.array_pta(kind=kind, seed=0)
    T, N, R = pta.get_basis(), pta.get_ndiag({}), pta.get_residuals()
    names = pta.param_names
    rind = [i for i, n in enumerate(names) if "rho" in n and "gw" in n]
    hind = np.array([i for i, n in enumerate(names) if "red" in n and "rho" in n])
    gwid = [np.arange(t.shape[1] - 60, t.shape[1]) for t in T]
    fixed = [np.full(t.shape[1] - 60, 1e-40) for t in T]
    red_col = hind.reshape(len(T), -1) if kind == "curn_red" else None
    sharded = shard == "pulsar" and world > 1
    hyper = None
    if kind == "curn_plred":
        # the reference's default redsample='mh' on per-pulsar power-law red noise (pta_gibbs.py:278-340),
        # aclength_hyper fixed (its warm-up's acor cannot run, pta_hyper); pulsar-sharded, every rank
        # applies its own pulsars' steps of the common step table and the (log10_A, gamma) values
        # travel in the [tau | x_red] all-gather (no other collective)
        from pulsar_timing_gibbsspec_amd.pta_hyper import HyperSpec
        hidx = np.array([i for i, n in enumerate(names) if "red" in n and ("log10_A" in n or "gamma" in n)])
        hyper = HyperSpec(pta, pta.params, [s for s in (pta.signals[k] for k in pta.signals) if "red" in s.name],
                          hidx, np.zeros(len(names)), 30, dev)
    if sharded:
        blocks = balanced_blocks(np.array([t.shape[1] ** 3 for t in T], float), world)
        lo, hi = blocks[rank]
        model = DeviceModel(ctx, T[lo:hi], N[lo:hi], R[lo:hi], gwid[lo:hi], fixed[lo:hi])
        rng = np.random.default_rng(0)
        x0 = rng.uniform(-9, -4, (C, len(names)))
        if hyper is not None:
            x0[:, hyper.hind] = rng.uniform(hyper.hlo_host, hyper.hhi_host, (C, hyper.n_h))
        ex = dict(allreduce=TauSumAllReduce()) if curn_mode == "sum" else \
            dict(gather=PulsarAllGather([np.arange(a, b) for a, b in blocks],
                                        ((2 if (red_col is not None or hyper is not None) else 1), 30, C),
                                        device=dev))
        eng = PTAChains(model, len(names), rind, red_col, (1e-18, 1e-8), (1e-20, 1e-8), C, x0,
                        P_global=len(T), psr_lo=lo, curn_mode=curn_mode, hyper=hyper,
                        hyper_acl=HYPER_ACL if hyper is not None else None, **ex)
    else:
        model = DeviceModel(ctx, T, N, R, gwid, fixed)
        rng = np.random.default_rng(rank)
        x0 = rng.uniform(-9, -4, (C, len(names)))
        if hyper is not None:
            x0[:, hyper.hind] = rng.uniform(hyper.hlo_host, hyper.hhi_host, (C, hyper.n_h))

        def make(nc):
            return PTAChains(model, len(names), rind, red_col, (1e-18, 1e-8), (1e-20, 1e-8), nc, x0[:nc],
                             chain_base=rank * C, curn_mode=curn_mode, hyper=hyper,
                             hyper_acl=HYPER_ACL if hyper is not None else None)
        eng = make(C)
    rec = torch.empty(K, C, len(names), dtype=torch.float64, device=dev)
    n_warm = warm(lambda: eng.sweep(x_rec=rec[0]), max(1, W))

    def run():
        for i in range(K):
            eng.sweep(x_rec=rec[i])
    el = timed_region(world, dev, run)
    if eng.info.cpu().numpy().any():
        raise RuntimeError("non-PD Sigma in the PTA bench")
    if curn_mode == "sum":
        eng.check_fx()
    total_chains = C if sharded else C * world
    value = total_chains * K / el
    out = dict(value=value, unit="chain-iters/s", ms_per_step=el / K * 1e3, steps=K,
               warmup={"n": n_warm, "unit": "sweeps", "min_ms": WARM_MS},
               chains_per_gpu=C, n_psr=len(T), n_param=len(names), n_gpus=world,
               scaling="strong" if sharded else "weak",
               sharding=("pulsars over %d GPUs (RCCL %s per sweep)" %
                         (world, "all-reduce of the tau sums" if curn_mode == "sum" else "all-gather of [tau | x_red]"))
               if sharded else "chains (no collective)")
    # roofline of the dominant kernels, each HIP-event timed alone on the context stream
    lib, h, m = ctx.lib, ctx.handle, eng.model
    st = ctx.stream
    ms_b = event_ms(st, lambda: eng._bdraw(None, _lib.EV_B, None), 5)
    b_shape = ctx.get_option(_lib.OPT_LAST_SWEEP_SHAPE)      # the tiled draw's kernel (cost model)
    mm = m.m.astype(float)
    bflop = C * float(np.sum(mm ** 3 / 3 + mm ** 2 / 2 + mm / 6 + 3 * mm ** 2))
    kernels = {"k_bdraw": dict(kernel_avg_ms=ms_b, bound="mfma", unit="TFLOP/s", peak=FP64_PEAK_TFLOPS,
                               achieved=bflop / (ms_b * 1e-3) / 1e12, alg_per_launch=bflop,
                               traffic=_ecorr_traffic(m.P * C, {"curn": "pmc_traffic_curn.json",
                                                                "curn_red": "pmc_traffic_red_bdraw.json",
                                                                "curn_plred": "pmc_traffic_plred_bdraw.json"}[kind])
                               if kind in ("curn", "curn_red", "curn_plred") else None,
                               name=("k_bdraw_pair (two chains per wave)" if b_shape == 3 else "k_bdraw_tiled")
                               if m.model_tiled is not None else "k_bdraw",
                               note="b|rho of every (pulsar, chain) system: sum_p m^3/3 + m^2/2 + m/6 + 3 m^2 "
                                    "flop per chain (SURVEY 8d)")}
    gp = grid_peak()
    n_f = eng.n_f
    if hyper is not None:
        hm = eng.hyper
        eng._update_irn()
        ms_seed = event_ms(st, lambda: (eng._gate_phiinv(with_gate=False, out=eng.phiinv_h, gate=eng._gate_h),
                                        hm.seed(eng.phiinv_h)), 5)
        x_save = eng.x.clone()
        ms_mh = event_ms(st, lambda: hm.steps(eng.x, HYPER_ACL, eng.it, eng.chain_base), 3)
        eng.x.copy_(x_save)
        nf = 60
        fl = nf ** 3 / 3 + nf ** 2 / 2 + nf / 6          # one NF x NF Schur-block factorisation
        # a pulsar-sharded rank evaluates only the steps of its own pulsars (expected share)
        own = float(np.mean((hm.hpsr >= 0).cpu().numpy()))
        kernels["k_hyper_mh"] = dict(
            kernel_avg_ms=ms_mh, bound="mfma", unit="TFLOP/s", peak=FP64_PEAK_TFLOPS,
            traffic=_ecorr_traffic(C, "pmc_traffic_hyper.json") if own == 1.0 else None,
            achieved=own * HYPER_ACL * C * fl / (ms_mh * 1e-3) / 1e12, alg_per_launch=own * HYPER_ACL * C * fl,
            own_step_share=own,
            note=f"{HYPER_ACL} single-parameter MH steps per chain (pta_gibbs.py:319-340), each one pulsar's "
                 "marginalised likelihood (NF x NF Schur block Cholesky, NF^3/3 + NF^2/2 + NF/6 flop; the "
                 "reference re-evaluates all 45 pulsars' full m x m systems per step)")
        kernels["k_bdraw"]["note"] += ("; with redsample='mh' the launch also writes lnL_p of every system "
                                       "(gs_ctx_set_bdraw_lnl: the red block's seed, likelihood mode for the "
                                       "systems the gate skips); the separate re-seed it replaces (phiinv + "
                                       "gs_lnlike_marg over every system) measures full_reseed_ms")
        kernels["k_bdraw"]["full_reseed_ms"] = ms_seed
    elif kind == "curn_red":
        check(lib, lib.gs_phi_from_x(h, C, n_f, _lib.ptr(eng.x), eng.n_param, _lib.ptr(eng.gw_col),
                                     _lib.ptr(eng.gwphi)))
        ms_r = event_ms(st, lambda: check(lib, lib.gs_rho_red(
            h, eng.P, C, n_f, _lib.ptr(eng.tau), _lib.ptr(eng.gwphi), eng.ngrid, _lib.ptr(eng.grid_red), None,
            eng.it, eng.chain_base, _lib.ptr(eng.x), eng.n_param, _lib.ptr(eng.red_col), None)), 5)
        # the rows the certified f32 pass could not prove and redid in f64 (one untimed launch)
        nfb = torch.zeros(1, dtype=torch.int32, device=eng.x.device)
        check(lib, lib.gs_ctx_set_grid_fallback_counter(h, _lib.ptr(nfb)))
        try:
            check(lib, lib.gs_rho_red(h, eng.P, C, n_f, _lib.ptr(eng.tau), _lib.ptr(eng.gwphi), eng.ngrid,
                                      _lib.ptr(eng.grid_red), None, eng.it, eng.chain_base, _lib.ptr(eng.x),
                                      eng.n_param, _lib.ptr(eng.red_col), None))
            torch.cuda.synchronize()
        finally:
            check(lib, lib.gs_ctx_set_grid_fallback_counter(h, None))
        ev = eng.P * n_f * C * eng.ngrid
        kernels["k_rho_red_cert16"] = dict(
            kernel_avg_ms=ms_r, bound="valu", unit="Geval/s", achieved=ev / (ms_r * 1e-3) / 1e9,
            alg_per_launch=ev, peak=valu_roof(*GRID_MIN_OPS["red"]) / 1e9,
            min_ops_per_unit=dict(zip(("plain", "transcendental"), GRID_MIN_OPS["red"])),
            op_mix_ceiling_f64_wave=(gp["red_evals_per_s"] / 1e9) if gp else None,
            f64_redo_rows_frac=int(nfb.item()) / (eng.P * n_f * C),
            traffic=_ecorr_traffic(C, "pmc_traffic_red.json"),
            alg_bytes_per_launch=eng.P * n_f * C * 24,
            note="grid-point evaluations ratio*exp(-ratio/2)*ln10 (pta_gibbs.py:265-266): P x n_f x C x 1000 "
                 "per launch (certified f32 pass, f64 redo of unproven rows: f64_redo_rows_frac); traffic: PMC "
                 "FETCH_SIZE x2 + WRITE_SIZE per launch (tools/archive/gpu_pmc_red.sh; algorithmic 24 B per row: tau, "
                 "irn and the x write) -- ~60 GB/s, far from the HBM roof; peak = "
                 "hardware VALU issue rate / the minimal op count per point in packed f32 (5 plain ops = 2.5 "
                 "v_pk_* slots at 4 cycles + rcp and exp at 8 per wave64: 26 cycles)")
        if not sharded:
            check(lib, lib.gs_phi_from_x(h, C, eng.PG * n_f, _lib.ptr(eng.x), eng.n_param, _lib.ptr(eng.red_col_g),
                                         _lib.ptr(eng.irn)))
            ms_c = event_ms(st, lambda: check(lib, lib.gs_rho_curn(
                h, eng.PG, C, n_f, _lib.ptr(eng.tau_g), _lib.ptr(eng.irn), eng.ngrid, _lib.ptr(eng.grid_gw), None,
                eng.it, eng.chain_base, _lib.ptr(eng.x), eng.n_param, _lib.ptr(eng.gw_col), None)), 5)
            ev = eng.PG * n_f * C * eng.ngrid
            kernels["k_rho_curn_fast"] = dict(
                kernel_avg_ms=ms_c, bound="valu", unit="Gterm/s", achieved=ev / (ms_c * 1e-3) / 1e9,
                alg_per_launch=ev, peak=valu_roof(*GRID_MIN_OPS["curn_term"]) / 1e9,
                min_ops_per_unit=dict(zip(("plain", "transcendental"), GRID_MIN_OPS["curn_term"])),
                op_mix_ceiling=(gp["curn_pulsar_terms_per_s"] / 1e9) if gp else None,
                note="(grid point, pulsar) terms of the common pdf product (pta_gibbs.py:192-205): "
                     "P x n_f x C x 1000 per launch; peak = hardware f64 VALU issue rate / 2 FMAs per term")
    else:
        def curn_sum():
            check(lib, lib.gs_rho_curn_sum(h, eng.PG, C, n_f, _lib.ptr(eng.S), eng.ngrid, _lib.ptr(eng.grid_gw), None,
                                           eng.it, eng.chain_base, _lib.ptr(eng.x), eng.n_param, _lib.ptr(eng.gw_col),
                                           None))
        nfb = torch.zeros(1, dtype=torch.int32, device=eng.x.device)
        check(lib, lib.gs_ctx_set_grid_fallback_counter(h, _lib.ptr(nfb)))
        try:
            curn_sum()
            torch.cuda.synchronize()
        finally:
            check(lib, lib.gs_ctx_set_grid_fallback_counter(h, None))
        ms_s = event_ms(st, curn_sum, 5)
        ev = n_f * C * eng.ngrid
        kernels["k_rho_curn_sum"] = dict(kernel_avg_ms=ms_s, bound="valu", unit="Geval/s",
                                         achieved=ev / (ms_s * 1e-3) / 1e9, alg_per_launch=ev,
                                         peak=valu_roof(*GRID_MIN_OPS["curn_sum"]) / 1e9,
                                         min_ops_per_unit=dict(zip(("plain", "transcendental"),
                                                                   GRID_MIN_OPS["curn_sum"])),
                                         op_mix_ceiling=(gp.get("curn_sum_evals_per_s", gp["red_evals_per_s"]) / 1e9)
                                         if gp else None,
                                         f64_redo_rows_frac=int(nfb.item()) / (n_f * C),
                                         note="n_f x C x 1000 grid points of the common pdf from the tau sums "
                                              "(certified f32 pass, f64 redo of unproven rows); peak = hardware "
                                              "VALU issue rate / the minimal op count per point (4 plain at 4 "
                                              "cycles + one exp at 8 per wave64)")
    for k in kernels.values():
        k["frac"] = (k["achieved"] / k["peak"]) if k.get("peak") else None
    dom = max(kernels, key=lambda k: kernels[k]["kernel_avg_ms"])
    out["roofline"] = dict(kernel=dom, **kernels[dom])
    out["kernels"] = kernels
    if not sharded and ess:
        # ESS per sweep of the common log10 rho from a separate untimed run of 256 chains from the
        # bench's start (gpu_ess: the CPU leg's run lengths and estimator), after the kernel timings
        # (its host-bound sweeps let the clock drop)
        out["ess"] = gpu_ess(sweep_block(make(min(C, 256)), rind), kind)
        out["ess_per_s"] = value * out["ess"]["per_chain_sweep_min_bin"]
    return out


def check(lib, rc):
    if rc != 0:
        raise RuntimeError(lib.gs_last_error().decode(errors="replace"))


def bench_indep(C, K, W, S, rank, world, dev, ess_on=True):
    """BASELINE configs[2]: the 45 simulated pulsars, each with its own 30-bin free
    spectrum (PulsarBlockGibbs per pulsar, pulsar_gibbs.py:620-710), C chains per pulsar,
    all (pulsar, chain) systems in one fused persistent launch per S sweeps.  N > 1:
    pulsars sharded over the ranks (contiguous blocks balanced by m^3), no collective;
    every rank's pulsars keep their global Philox index (bit-identical to N = 1)."""
    from pulsar_timing_gibbsspec_amd import _lib, synthetic
    from pulsar_timing_gibbsspec_amd.array_gibbs import shard_pulsars
    from pulsar_timing_gibbsspec_amd.engine import DeviceModel, FreeSpectrumChains
    ptas = synthetic.pulsar_ptas(synthetic.array_pta(kind="indep", seed=0))
    lo, hi = shard_pulsars(ptas, rank, world) if world > 1 else (0, len(ptas))
    mine = ptas[lo:hi]
    T = [p.get_basis()[0] for p in mine]
    ctx = _lib.Context(dev.index, seed=20251019)
    ctx.set_option(_lib.OPT_PSR_BASE, lo)
    model = DeviceModel(ctx, T, [p.get_ndiag({})[0] for p in mine], [p.get_residuals()[0] for p in mine],
                        [np.arange(60)] * len(T), [np.full(t.shape[1] - 60, 1e-40) for t in T])
    P = len(T)
    x0 = np.random.default_rng(0).uniform(-9, -4, (len(ptas) * C, 30))[lo * C:hi * C]
    run = FreeSpectrumChains(model, 1e-18, 1e-8, C, x0)
    x_rec = torch.empty(S, P * C, 30, dtype=torch.float64, device=dev)
    b_rec = torch.empty(S, P * C, model.ldb, dtype=torch.float64, device=dev)
    n_warm = warm(lambda: run.run(S, x_rec=x_rec[:S], b_rec=b_rec[:S]), 1) if W else 0  # full launches
    torch.cuda.synchronize()
    launches = []

    def go():
        done = 0
        while done < K:
            n = min(S, K - done)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(ctx.stream)
            run.run(n, x_rec=x_rec[:n], b_rec=b_rec[:n])
            e1.record(ctx.stream)
            launches.append((e0, e1, n))
            done += n
    el = timed_region(world, dev, go)
    kname = sweep_kernel(ctx, rm=model.NMX > 16)     # the timed launches' shape (before the ESS run's)
    if run.info.cpu().numpy().any():
        raise RuntimeError("non-PD Sigma in the configs[2] bench")
    ms = np.array([a.elapsed_time(b) for a, b, _ in launches])
    sw = np.array([n for _, _, n in launches])
    per_sweep = float(np.sum(ms) / 1e3 / np.sum(sw))
    mm = model.m.astype(float)
    flops_sweep = C * float(np.sum(mm ** 3 / 3 + mm ** 2 / 2 + mm / 6 + 3 * mm ** 2))
    ach = flops_sweep / per_sweep / 1e12
    # ESS per sweep, min over (pulsar, bin): a separate untimed run of CE chains per pulsar (gpu_ess)
    CE = min(C, 64)
    ess_run = FreeSpectrumChains(model, 1e-18, 1e-8, CE, np.random.default_rng(1).uniform(-9, -4, (P * CE, 30)))
    xe = torch.empty(S, P * CE, 30, dtype=torch.float64, device=dev)

    def block(n_max, rec):
        n = min(S, n_max)
        ess_run.run(n, record_b=False, x_rec=xe[:n])
        return n, (xe[:n].view(n, P, CE, 30).permute(0, 2, 1, 3).reshape(n, CE, P * 30) if rec else None)
    ess = gpu_ess(block, "indep") if ess_on else None
    del ess_run, xe
    return dict(value=C * K / el, unit="array-iters/s", ms_per_step=el / K * 1e3, steps=K,
                warmup={"n": n_warm, "unit": "launches", "min_ms": WARM_MS},
                chains_per_pulsar=C, n_psr=len(ptas), n_psr_local=P, m_range=[int(model.m.min()), int(model.m.max())],
                n_gpus=world, scaling="strong" if world > 1 else "weak",
                sharding=(f"pulsars over {world} GPUs (no collective)" if world > 1 else "one GPU"),
                pulsar_iters_per_s=C * K * len(ptas) / el,
                ess_per_s=C * K / el * ess["per_chain_sweep_min_bin"] if ess else None, ess=ess,
                roofline={"kernel": kname,
                          "bound": "mfma", "unit": "TFLOP/s", "achieved": ach,
                          "peak": FP64_PEAK_TFLOPS, "frac": ach / FP64_PEAK_TFLOPS,
                          "kernel_avg_ms": per_sweep * S * 1e3, "sweeps_per_launch": S,
                          "alg_flops_per_launch": flops_sweep * S,
                          "traffic": _ecorr_traffic(P * C, "pmc_traffic_indep.json") if S == 100 else None,
                          "alg_bytes_per_launch": P * C * S * 8 * (30 + model.ldb),
                          "note": "sum over the rank's pulsars of m^3/3 + m^2/2 + m/6 + 3 m^2 flop per chain-sweep "
                                  "(SURVEY 8d) x C x S over the HIP-event launch time; traffic: PMC of the largest "
                                  "launch (profiles/pmc_traffic_indep.json), alg_bytes: the x and b rows recorded"})


def bench_config5(C, K, W, rank, world, dev, n_psr=200, n_toa=10_000, n_f=100, aclength=20, reps=5, ess_on=True):
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
    n_warm = warm(eng.sweep, W)
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
    # ESS per sweep of log10 rho: an untimed run of 64 chains on the CPU leg's pulsar
    # (config5_array(n_psr=1, seed=1), oracle/cpu_baseline.py config5), same start x0
    ess = None
    if ess_on:
        d1 = synthetic.config5_array(n_psr=1, n_toa=n_toa, n_f=n_f, seed=1)
        wm1 = WhiteNoiseModel(ctx, d1["T"], d1["r"], d1["sigma"], d1["backend"], [d1["fidx"]], [d1["phiinv_fixed"]],
                              [d1["white"]], 64)
        e1n = WhiteArrayChains(wm1, d1["n_param"], d1["gw_cols"], d1["rhomin"], d1["rhomax"],
                               np.repeat(d1["x0"], 64, axis=0), aclength=aclength, chain_base=rank * 64)
        ess = gpu_ess(sweep_block(e1n, d1["gw_cols"]), "config5")
        del e1n, wm1, d1
    n_sys = n_psr * C
    flops = n_sys * (n_toa * m * (m + 1) + 2 * n_toa * m)      # SYRK + TNr per system
    tflops = flops / (refresh_ms * 1e-3) / 1e12
    return dict(value=C * world * K / el, unit="chain-iters/s", ms_per_step=el / K * 1e3, steps=K,
                warmup={"n": n_warm, "unit": "sweeps", "min_ms": WARM_MS},
                ess_per_s=C * world * K / el * ess["per_chain_sweep_min_bin"] if ess else None, ess=ess,
                chains_per_gpu=C, n_psr=n_psr, n_toa=n_toa, m=m, aclength=aclength,
                roofline={"bound": "mfma", "kernel": "k_white_syrk + k_prefix (gs_white_tnt + gs_prefix_sys)",
                          "achieved": tflops, "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                          "frac": tflops / FP64_PEAK_TFLOPS, "kernel_avg_ms": refresh_ms,
                          "alg_flops_per_launch": flops,
                          "traffic": _ecorr_traffic(C, "pmc_traffic_syrk.json") if n_psr == 200 else None,
                          "note": "per-chain TNT/d of all 200 pulsars (n m (m+1) + 2 n m flop per system) "
                                  "over the HIP-event time of one refresh (SYRK + prefix)"})


def _ecorr_traffic(C, fname="pmc_traffic_ecorr.json"):
    """HBM bytes per launch of k_ecorr_prefix<likelihood> from the committed PMC passes
    (tools/archive/gpu_pmc_ecorr.sh -> profiles/pmc_traffic_ecorr.json for the shared-operand kernel,
    profiles/pmc_traffic_ecorr_white.json for the per-chain-operand one), same chain count only."""
    try:
        d = json.load(open(os.path.join(ROOT, "profiles", fname)))
    except (OSError, ValueError):
        return None
    return d.get("bytes_per_launch") if d.get("chains") == C else None


def ecorr_step_roofline(ctx, em, x, phiinv_F, reps=10, traffic_file="pmc_traffic_ecorr_step.json"):
    """The ECORR Metropolis step's kernel (gs_ecorr_lnl_state, incremental: the moved backend's epochs
    only), HIP-event timed alone on the context stream: a full evaluation stores the state at x, one
    proposal (gs_ecorr_propose, step 0) is drawn, then `reps` steps from that state (the state slot is
    not adopted, so every step reads the same T).  Algorithmic flops per chain: the moved backend's
    epochs (n_E / n_backends on average) x (mR+1)(mR+2) + nM (NF+1)(NF+2) + (NF+1)^3/3."""
    from pulsar_timing_gibbsspec_amd._lib import check as lcheck, ptr
    if not (em.incremental and em.fused and em.fused_lnl):
        return None
    em._state_buffers()
    em.tidx.zero_()
    em._eval_state(x, phiinv_F)
    lcheck(ctx.lib.gs_ecorr_propose(ctx.handle, em.C, em.n_bk, ptr(em.ecol), ptr(em.emin), ptr(em.emax), ptr(x),
                                    x.shape[1], em.n_param, ptr(em.xq), 0, 0, 0, None, ptr(em.prop)),
           "gs_ecorr_propose")
    for _ in range(3):
        em._eval_state(em.xq, phiinv_F, x_old=x)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(ctx.stream)
    for _ in range(reps):
        em._eval_state(em.xq, phiinv_F, x_old=x)
    e1.record(ctx.stream)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    mR, NF, nM, C = em.mR, em.NF, em.nm, em.C
    flops = C * (em.ne / em.n_bk * (mR + 1) * (mR + 2) + nM * (NF + 1) * (NF + 2) + (NF + 1) ** 3 // 3)
    nb = em.ldbp // 16
    tfl = flops / (ms * 1e-3) / 1e12
    state = C * 2 * 8 * 256 * nb * (nb + 1) // 2
    traffic = _ecorr_traffic(C, traffic_file)
    return {"kernel": "k_ecorr_prefix<likelihood mode, incremental step> (gs_ecorr_lnl_state)", "bound": "mfma",
            "achieved": tfl, "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s", "frac": tfl / FP64_PEAK_TFLOPS,
            "kernel_avg_ms": ms, "alg_flops_per_launch": flops, "traffic": traffic,
            "state_bytes_per_launch": state, "traffic_over_state": (traffic / state) if traffic else None,
            "hbm_gbs": (traffic / (ms * 1e-3) / 1e9) if traffic else None,
            "note": "the per-step kernel of the ECORR Metropolis block (aclength launches per sweep; the full "
                    "evaluation runs once per block): the moved backend's epochs re-weighted from the stored "
                    "T = Ap - P (read and the proposal's written: state_bytes_per_launch); traffic = PMC "
                    "FETCH_SIZE x2 + WRITE_SIZE of the bench's own step launches (profiles/r06d, r06e, "
                    "tools/pmc_ecorr_r06.py)"}


def bench_ecorr_white(C, K, W, rank, world, dev, aclength=10, ess_on=True):
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
    n_warm = warm(eng.sweep, W)
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
    step = ecorr_step_roofline(ctx, em, eng.x, eng.phiinv_F, traffic_file="pmc_traffic_ecorr_white_step.json")
    mR, NF, nM = em.mR, em.NF, em.nm
    flops = C * (ne * (mR + 1) * (mR + 2) + nM * (NF + 1) * (NF + 2) + (NF + 1) ** 3 // 3)
    tflops = flops / (k_ms * 1e-3) / 1e12
    # algorithmic HBM bytes of one launch: every chain's own operands, read once -- the [B | d_E]
    # rows (ne x ldbx), the upper 16x16 tiles of Ap (nb (nb + 1) / 2 of them, nb = ldbx / 16),
    # the epoch diagonal, phiinv_F -- and lnl + aux written
    nb = em.ldbx // 16
    alg_bytes = C * 8 * (ne * em.ldbx + 256 * nb * (nb + 1) // 2 + ne + NF + 5)
    traffic = _ecorr_traffic(C, "pmc_traffic_ecorr_white.json")
    value = C * world * K / el
    ess = gpu_ess(sweep_block(eng, gw, 256), "ecorr_white") if ess_on else None   # the chains continued, untimed
    return dict(value=value, unit="chain-iters/s", ms_per_step=el / K * 1e3, steps=K,
                warmup={"n": n_warm, "unit": "sweeps", "min_ms": WARM_MS},
                ess_per_s=value * ess["per_chain_sweep_min_bin"] if ess else None, ess=ess,
                chains_per_gpu=C, m=m, n_epoch=ne, aclength_white=aclength, aclength_ecorr=aclength,
                roofline={"bound": "mfma", "kernel": "k_ecorr_prefix<likelihood mode, per-chain operands>",
                          "achieved": tflops, "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                          "frac": tflops / FP64_PEAK_TFLOPS, "kernel_avg_ms": k_ms, "alg_flops_per_launch": flops,
                          "traffic": traffic, "alg_bytes_per_launch": alg_bytes,
                          "traffic_over_alg": (traffic / alg_bytes) if traffic else None,
                          "hbm_frac": alg_bytes / (k_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                          "note": "as the ecorr line; each chain's own [B | d_E] rows and Ap tiles stream from "
                                  "HBM (alg_bytes_per_launch); traffic = PMC FETCH_SIZE x2 + WRITE_SIZE of the "
                                  "bench's own launches (profiles/r06d, r06e; tools/pmc_ecorr_r06.py); the full "
                                  "evaluation (once per Metropolis block); the per-step kernel: step_roofline"},
                step_roofline=step,
                config="SURVEY 8f-4 with EFAC/EQUAD sampled: J1713-like pulsar, 2 backends, 136 ECORR epochs, "
                       "white MH + per-chain TNT + ECORR MH + analytic rho|b + gated b per sweep, chain-sharded")


def bench_ecorr(C, K, W, rank, world, dev, aclength=10, reps=10, ess_on=True):
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
    n_warm = warm(eng.sweep, W)
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
    step = ecorr_step_roofline(ctx, em, eng.x, eng.phiinv_F)
    mR, NF, nM = em.mR, em.NF, em.nm
    # epoch-weighted SYRK (lower triangle of [B | d_E]^T W [B | d_E]) + the fixed-prior Schur
    # update + the (NF+1)-augmented Cholesky of the free-spectrum block
    flops = C * (ne * (mR + 1) * (mR + 2) + nM * (NF + 1) * (NF + 2) + (NF + 1) ** 3 // 3)
    tflops = flops / (k_ms * 1e-3) / 1e12
    value = C * world * K / el
    ess = gpu_ess(sweep_block(eng, gw, 256), "ecorr") if ess_on else None   # the chains continued, untimed
    return dict(value=value, unit="chain-iters/s", ms_per_step=el / K * 1e3, steps=K,
                warmup={"n": n_warm, "unit": "sweeps", "min_ms": WARM_MS},
                ess_per_s=value * ess["per_chain_sweep_min_bin"] if ess else None, ess=ess,
                chains_per_gpu=C, m=m, n_epoch=ne, m_R=mR, aclength=aclength,
                roofline={"bound": "mfma", "kernel": ("k_ecorr_prefix<likelihood mode>" if em.fused and em.fused_lnl
                                                      else "k_ecorr_schur + k_prefix + k_lnlike_marg"),
                          "achieved": tflops,
                          "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s", "frac": tflops / FP64_PEAK_TFLOPS,
                          "kernel_avg_ms": k_ms, "alg_flops_per_launch": flops,
                          "traffic": _ecorr_traffic(C),
                          "note": "ne (mR+1)(mR+2) + nM (NF+1)(NF+2) + (NF+1)^3/3 flop per chain (epoch-weighted "
                                  "SYRK with the d_E row + fixed-prior Schur update + F-block Cholesky) over the "
                                  "HIP-event time of one all-chain likelihood launch; traffic: PMC FETCH_SIZE x2 + "
                                  "WRITE_SIZE of the bench's own launches (profiles/r06d, r06e; operands "
                                  "L2-resident); the full evaluation (once per Metropolis block); the per-step "
                                  "kernel: step_roofline"},
                step_roofline=step,
                config="SURVEY 8f-4: J1713-like pulsar, basis ECORR (2 backends, 136 epochs) + 30-bin free "
                       "spectrum + 16-col TM, ECORR MH + analytic rho|b + gated b per sweep, chain-sharded")


LINE_MAX = 8192            # the driver parses stdout's last line; round 5's 22.9 KB line did not parse


def _sig(v, n=5):
    """A float rounded to n significant digits (ints, None and strings unchanged)."""
    if isinstance(v, float) and v == v and v not in (float("inf"), float("-inf")) and v != 0.0:
        return float(f"{v:.{n}g}")
    return v


def _pick(d, keys, n=5):
    return {k: _sig(d[k], n) for k in keys if isinstance(d, dict) and d.get(k) is not None}


def _cpu_brief(c, full=False):
    if not c:
        return None
    b = _pick(c, ("value", "unit", "cores", "kind", "per_process", "ess_per_s", "error"))
    if full and c.get("sample"):
        b["sample"] = c["sample"]
    if (c.get("reference_equivalent") or {}).get("value"):
        b["reference_equivalent"] = _sig(c["reference_equivalent"]["value"])
    e = c.get("ess") or {}
    if e.get("ess_per_sweep") is not None:
        b["ess_per_sweep"] = _pick(e, ("ess_per_sweep", "se", "chains", "sweeps", "burn_in"))
    return b


def _ess_brief(e):
    return _pick(e or {}, ("per_chain_sweep_min_bin", "se", "bin", "chains", "sweeps", "burn_in", "z_vs_cpu"))


def result_line(out):
    """The ONE stdout JSON line: the contract's keys, the headline's roofline / cpu_baseline / ESS,
    and per secondary line only {value, ms_per_step, ess, roofline frac + kernel time, traffic
    ratio, cpu value}.  Notes, per-kernel tables and calibration text go to the detail file
    (bench_detail.json).  Kept under LINE_MAX bytes (tests/test_bench_line.py)."""
    keys = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
            "vs_baseline", "dtype", "data", "config", "ess_per_s")
    line = {k: out.get(k) for k in keys}
    line["ess"] = _ess_brief(out.get("ess"))
    rf = out.get("roofline") or {}
    line["roofline"] = _pick(rf, ("bound", "achieved", "peak", "unit", "frac", "traffic", "kernel", "kernel_avg_ms",
                                  "alg_flops_per_launch", "executed_frac"), 6)
    si = rf.get("simd_issue") or {}
    if si:
        line["roofline"]["simd_issue"] = _pick(si, ("frac", "valu_per_draw", "mfma_per_draw", "source"))
    line["cpu_baseline"] = _cpu_brief(out.get("cpu_baseline"), full=True)
    hs = out.get("with_host_stream")
    if hs:
        line["with_host_stream"] = dict(_pick(hs, ("value", "ms_per_step")),
                                        all_b=_pick(hs.get("all_b") or {}, ("value", "ms_per_step")))
    sec = {}
    for name, d in (out.get("secondary") or {}).items():
        s = _pick(d, ("value", "unit", "ms_per_step", "ess_per_s", "n_gpus", "scaling"))
        if d.get("ess"):
            s["ess"] = _ess_brief(d["ess"])
        r = d.get("roofline") or {}
        s["roofline"] = _pick(r, ("kernel", "frac", "kernel_avg_ms", "traffic_over_alg"))
        if r.get("traffic") and r.get("alg_bytes_per_launch") and "traffic_over_alg" not in s["roofline"]:
            s["roofline"]["traffic_over_alg"] = _sig(r["traffic"] / r["alg_bytes_per_launch"])
        if d.get("step_roofline"):
            s["step_roofline"] = _pick(d["step_roofline"], ("frac", "kernel_avg_ms", "traffic_over_state"))
        if d.get("cpu_baseline"):
            s["cpu_baseline"] = _cpu_brief(d["cpu_baseline"])
        sec[name] = s
    line["secondary"] = sec
    if out.get("detail"):
        line["detail"] = out["detail"]
    txt = json.dumps(line, separators=(",", ":"))
    if len(txt) > LINE_MAX:                     # last resort: the headline alone still parses
        line["secondary"] = {k: _pick(v, ("value", "ms_per_step", "ess_per_s")) for k, v in sec.items()}
        txt = json.dumps(line, separators=(",", ":"))
    return txt


def write_detail(out, path=None):
    """The full record (every note, kernel table, calibration and ESS per bin) beside the line."""
    path = path or os.environ.get("GS_BENCH_DETAIL") or os.path.join(ROOT, "gpurun_out", "bench_detail.json")
    try:
        os.makedirs(os.path.dirname(path), exist_ok=True)
        with open(path, "w") as f:
            json.dump(out, f, indent=1, default=str)
        return os.path.relpath(path, ROOT)
    except OSError:
        return None


def launch_ranks(args_list, n):
    """`bench.py --gpus N` outside a launcher: start N ranks of this script under
    torch.distributed.run (one process per GPU, 127.0.0.1 rendezvous) and return their
    exit code.  Runs before anything here touches the GPU; the ranks are child
    processes, nothing is exec'd."""
    import socket
    import subprocess
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + args_list
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


_PHASE = ["start"]


def phase(name):
    """Progress marker on stderr (stdout carries only the result line)."""
    _PHASE[0] = name
    print(f"[bench] {name}", file=sys.stderr, flush=True)


def _heartbeat(period=30.0):
    """A line on stderr every ``period`` seconds while the bench runs, so a supervisor that takes a
    silent command for a hung one (no output for minutes) sees the CPU-baseline and ESS phases --
    several minutes of host work with nothing else to print -- as alive."""
    import threading
    t0 = time.time()

    def run():
        while True:
            time.sleep(period)
            print(f"[bench] ... {_PHASE[0]} ({time.time() - t0:.0f} s)", file=sys.stderr, flush=True)
    threading.Thread(target=run, daemon=True).start()


def main():
    _heartbeat()
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20, help="headline steps = fused 100-sweep launches")
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--ess", type=int, default=1, help="measure ESS per sweep on the GPU (untimed runs, "
                    "diagnostics.ESS_RUN lengths) and, with the CPU baseline, on the CPU port too (1/0)")
    ap.add_argument("--chains", type=int, default=4096, help="chains per GPU")
    ap.add_argument("--sweeps-per-launch", type=int, default=100)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=8.0, help="seconds per CPU-baseline process")
    ap.add_argument("--cpu-ess-procs", type=int, default=12, help="CPU ESS chains run at once beside the GPU "
                    "work (oracle.cpu_baseline.ESS_CHAINS independent single-thread chains per line, EssPool)")
    ap.add_argument("--bcast", type=int, default=None, help="GS_OPT_BCAST (0 readlane, 1 LDS, 2 batched, 3 tile)")
    ap.add_argument("--sched", type=int, default=None,
                    help="GS_OPT_SWEEP_SCHED for the headline (0 cost model, 1 hand-off, 2 one chain per wave, "
                         "3 two chains per wave)")
    ap.add_argument("--host-stream", type=int, default=1,
                    help="also time the headline with every recorded row streamed to pinned host memory (1/0)")
    ap.add_argument("--indep", type=int, default=1, help="measure BASELINE configs[2] (45 independent pulsars)")
    ap.add_argument("--indep-chains", type=int, default=256, help="chains per pulsar for configs[2]")
    ap.add_argument("--indep-steps", type=int, default=500)
    ap.add_argument("--pta", default="curn_red,curn,curn_plred", help="secondary PTA configs measured in the "
                    "same run (comma list of curn_red, curn, curn_plred; or none). curn uses the sufficient-statistic "
                    "draw; curn_plred the red-noise Metropolis block (redsample='mh')")
    ap.add_argument("--pta-chains", type=int, default=2048,
                    help="chains per GPU for the PTA lines (measured: 256 -> 1024 -> 2048 -> 4096 chains give "
                         "CURN + red 3.0e5 -> 3.8e5 -> 3.9e5 -> 4.0e5 chain-it/s: saturated at 2048)")
    ap.add_argument("--pta-steps", type=int, default=200)
    ap.add_argument("--config5", type=int, default=1, help="measure BASELINE configs[4] too (1/0)")
    ap.add_argument("--ecorr", type=int, default=1, help="measure the basis-ECORR path (SURVEY 8f-4) too (1/0)")
    ap.add_argument("--ecorr-chains", type=int, default=4096)
    ap.add_argument("--ecorr-steps", type=int, default=10)
    ap.add_argument("--c5-chains", type=int, default=16)
    ap.add_argument("--c5-steps", type=int, default=5)
    ap.add_argument("--dry-run", action="store_true", help="launcher/rendezvous check only: no GPU work")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(sys.argv[1:], args.gpus))

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # one process per GPU over RCCL; GS_DIST_BACKEND=gloo (and more ranks than GPUs, ranks
    # sharing devices round-robin) only to rehearse the multi-rank paths on one GPU
    backend = os.environ.get("GS_DIST_BACKEND", "nccl")
    if args.dry_run:
        if world > 1:
            dist.init_process_group("gloo")
            world = dist.get_world_size()
        if rank == 0:
            print(json.dumps({"dry_run": True, "n_gpus": world, "gpus_requested": args.gpus}), flush=True)
        if world > 1:
            dist.destroy_process_group()
        return
    if backend != "nccl":
        local = local % torch.cuda.device_count()
    if world > 1:
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
        world = dist.get_world_size()          # the ranks the process group actually holds
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    cpu = not args.no_cpu_baseline and world == 1 and rank == 0   # rank 0 at N = 1 only
    # the CPU port's ESS per sweep: one single-process run per chain-mixing config, started now so
    # it runs beside the GPU work (numpy only, one thread each); the throughput processes of
    # cpu_baseline run at the very end, after these have finished, so nothing competes with them
    pool = None
    if cpu and args.ess:
        from oracle.cpu_baseline import EssPool
        pool = EssPool(args.cpu_ess_procs, os.path.join(ROOT, "gpurun_out", "ess_rows"))
        # slowest first, so the longest chains start while the GPU lines run
        lines = [k for k in ("curn_red", "curn_plred", "curn") if k in args.pta.split(",")]
        lines += (["config5"] if args.config5 else []) + (["indep"] if args.indep else [])
        lines += (["ecorr_white", "ecorr"] if args.ecorr else []) + ["single"]
        for kind in lines:
            pool.submit(kind)

    phase("headline configs[1]")
    from pulsar_timing_gibbsspec_amd import _lib, synthetic
    from pulsar_timing_gibbsspec_amd.engine import DeviceModel, FreeSpectrumChains, HistoryStreamer

    pta = synthetic.single_pulsar_pta("J1713+0747", seed=0)
    T, N, r = pta.get_basis()[0], pta.get_ndiag({})[0], pta.get_residuals()[0]
    gwid = np.arange(60)
    ctx = _lib.Context(local, seed=20251015)
    if args.bcast is not None:
        ctx.set_option(_lib.OPT_BCAST, args.bcast)
    if args.sched is not None:
        ctx.set_option(_lib.OPT_SWEEP_SCHED, args.sched)
    model = DeviceModel(ctx, [T], [N], [r], [gwid], [np.full(T.shape[1] - 60, 1e-40)])
    C = args.chains
    x0 = np.random.default_rng(rank).uniform(-9, -4, (C, 30))
    run = FreeSpectrumChains(model, 1e-18, 1e-8, C, x0, chain_base=rank * C)
    K, W, S = args.steps, args.warmup, max(1, args.sweeps_per_launch)
    m = int(model.m[0])
    # one launch's history block in HBM, rewritten by every launch (the rows a save block holds)
    x_rec = torch.empty(S, C, 30, dtype=torch.float64, device=dev)
    b_rec = torch.empty(S, C, model.ldb, dtype=torch.float64, device=dev)

    for _ in range(W):                                # warmup (untimed)
        run.run(S, x_rec=x_rec, b_rec=b_rec)
    stream = ctx.stream
    evs = []

    def headline():
        for _ in range(K):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            run.run(S, x_rec=x_rec, b_rec=b_rec)
            e1.record(stream)
            evs.append((e0, e1))
    el = timed_region(world, dev, headline)
    kname = sweep_kernel(ctx)                        # the timed launches' shape (before the ESS run's)
    info = run.info.cpu().numpy()
    if info.any():
        raise RuntimeError(f"{int((info != 0).sum())} chains hit a non-PD Sigma")

    total_chains = C * world
    value = total_chains * K * S / el
    # roofline of the fused sweep kernel (dominant kernel: one launch per step of S sweeps)
    kern_ms = np.array([a.elapsed_time(b) for a, b in evs])
    launch_s = float(np.mean(kern_ms)) / 1e3
    alg_flops_launch = flops_per_chain_sweep(m) * C * S
    achieved = alg_flops_launch / launch_s / 1e12
    exe = executed_flops_per_chain_sweep(model.NF, int(model.nm[0])) * C * S / launch_s / 1e12
    # ESS per chain-sweep from a separate untimed run of 256 chains (same kernel, same law; gpu_ess:
    # the CPU leg's run lengths and estimator)
    ce = min(C, 256)
    ess_run = FreeSpectrumChains(model, 1e-18, 1e-8, ce, x0[:ce], chain_base=rank * C)
    xe = torch.empty(S, ce, 30, dtype=torch.float64, device=dev)

    def ess_block(n_max, rec):
        n = min(S, n_max)
        ess_run.run(n, record_b=False, x_rec=xe[:n])
        return n, (xe[:n] if rec else None)
    ess_rec = gpu_ess(ess_block, "single") if args.ess else None
    ess = value * ess_rec["per_chain_sweep_min_bin"] if ess_rec else None
    del xe, ess_run
    K_sweeps = K * S

    host = None
    if args.host_stream:
        # the same K sweeps as PulsarBlockGibbs.sample runs them: each block's recorded rows go
        # to pinned host memory on a side stream while the next block computes.  sample()'s
        # default for 4096 chains streams x of every chain and b of chain 0 (the reference's
        # bchain); with record_bchains=True every chain's b too.
        def streamed_rate(bk, direct):
            streamer = HistoryStreamer(ctx, [(S, C, 30), (S, bk, model.ldb)], direct=direct)

            def go():
                done, slot, pending = 0, 0, None
                while done < K_sweeps:
                    n = min(S, K_sweeps - done)
                    xr, br = streamer.buffers(slot, n)
                    run.run(n, x_rec=xr, b_rec=br, record_b_chains=bk)
                    streamer.submit(slot, n)
                    if pending is not None:
                        streamer.fetch(pending)
                    pending, slot, done = slot, slot ^ 1, done + n
                if pending is not None:
                    streamer.fetch(pending)
            el_h = timed_region(world, dev, go)
            return total_chains * K_sweeps / el_h, el_h / K * 1e3
        v0, ms0 = streamed_rate(1, [True, True])
        v1, ms1 = streamed_rate(C, [True, False])
        host = {"value": v0, "unit": "chain-iters/s", "ms_per_step": ms0,
                "bytes_per_step": S * (C * 30 * 8 + model.ldb * 8),
                "note": "sample()'s default: the kernel writes x of every chain and b of chain 0 (the reference's "
                        "bchain, GS_OPT_BREC_CHAINS = 1) straight into pinned host memory (zero-copy over PCIe), "
                        "read while the next block runs (engine.HistoryStreamer)",
                "all_b": {"value": v1, "ms_per_step": ms1, "bytes_per_step": C * (30 + model.ldb) * 8,
                          "note": "record_bchains=True: every chain's b as well (HBM, then the copy engine)"}}

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
                       "step": f"one fused launch of {S} sweeps of every chain", "sweeps_per_step": S,
                       "bcast": ctx.get_option(_lib.OPT_BCAST),
                       "parallelism": f"chains sharded over {world} GPU(s), no collective"},
            "ess_per_s": ess,
            "ess": ess_rec,
            "roofline": {"bound": "mfma", "achieved": achieved, "peak": FP64_PEAK_TFLOPS,
                         "unit": "TFLOP/s", "frac": achieved / FP64_PEAK_TFLOPS,
                         "traffic": pmc_traffic(S, C),
                         "kernel": kname, "kernel_avg_ms": launch_s * 1e3,
                         "alg_flops_per_launch": alg_flops_launch,
                         "note": "achieved = SURVEY 8d's algorithmic flops (dense m=76 potrf + 3 solves); the kernel "
                                 "executes fewer (executed_*: NF=60 Schur block after the fixed-prior prefix)",
                         "executed_tflops": exe, "executed_frac": exe / FP64_PEAK_TFLOPS,
                         "simd_issue": simd_issue(launch_s, C * S)},
            "with_host_stream": host,
        }
    sec = {}
    cpu_kinds = {}

    def add(name, d, kind=None):
        if rank == 0:
            if kind:
                cpu_kinds[name] = kind
            sec[name] = d

    if args.indep:
        phase("configs[2] indep")
        d = bench_indep(args.indep_chains, args.indep_steps, 2, 100, rank, world, dev, ess_on=bool(args.ess))
        d["config"] = ("configs[2]: 45 simulated pulsars, each its own 30-bin free spectrum (m 68..77), "
                       f"{args.indep_chains} chains per pulsar, one fused launch per 100 sweeps")
        add("indep", d, "indep")
    for kind in [k for k in args.pta.split(",") if k and k != "none"]:
        phase(f"configs[3] {kind}")
        d = bench_pta(kind, args.pta_chains, args.pta_steps, 2, rank, world, dev, ctx, shard="chain",
                      ess=bool(args.ess))
        d["config"] = (f"configs[3]: 45-pulsar CURN{' + per-pulsar red' if kind == 'curn_red' else ''} free "
                       f"spectrum, common draw {'from the tau sums' if kind == 'curn' else 'exact product'}")
        if kind == "curn_plred":
            d["config"] = ("configs[3] with the reference's default redsample='mh': 45-pulsar CURN free spectrum + "
                           f"per-pulsar power-law red noise by {HYPER_ACL} Metropolis steps per sweep")
        add(kind, d, kind)
        if world > 1:
            d = bench_pta(kind, args.pta_chains, args.pta_steps, 2, rank, world, dev, ctx, shard="pulsar", ess=False)
            d["config"] = f"configs[3] {kind}, pulsars sharded over the ranks with the per-sweep RCCL exchange"
            add(kind + "_pulsar_sharded", d)
    if args.ecorr:
        phase("ecorr")
        d = bench_ecorr(args.ecorr_chains, args.ecorr_steps, 2, rank, world, dev, ess_on=bool(args.ess))
        d.update(sharding="chains (no collective)", scaling="weak", n_gpus=world)
        add("ecorr", d, "ecorr")
        d = bench_ecorr_white(args.ecorr_chains, args.ecorr_steps, 2, rank, world, dev, ess_on=bool(args.ess))
        d.update(sharding="chains (no collective)", scaling="weak", n_gpus=world)
        add("ecorr_white", d, "ecorr_white")
    if args.config5:
        phase("configs[4] config5")
        d = bench_config5(args.c5_chains, args.c5_steps, 1, rank, world, dev, ess_on=bool(args.ess))
        d.update(n_gpus=world, scaling="weak", sharding="chains (no collective)")
        d["config"] = ("configs[4]: 200 synthetic pulsars x 10^4 TOAs x 100 frequencies (m=216), "
                       "white-noise MH (20 steps) + per-chain TNT recompute every sweep, chain-sharded")
        add("config5", d, "config5")
    if rank == 0 and cpu:
        phase("cpu baseline (ESS runs, then one single-thread process per core per line)")
        from pulsar_timing_gibbsspec_amd.diagnostics import ess_compare
        ess_cpu = {}
        if pool is not None:
            for kind in ["single"] + list(cpu_kinds.values()):
                ess_cpu[kind] = pool.collect(kind)
        calib = cpu_calibration()

        def baseline(kind, gpu_ess_rec):
            b = cpu_line(kind, args.cpu_seconds)
            e = ess_cpu.get(kind)
            if e is not None:
                b["ess"] = e
                if b.get("value") and "ess_per_sweep" in e:
                    b["ess_per_s"] = b["value"] * e["ess_per_sweep"]
                if gpu_ess_rec and "per_bin" in e:
                    cmp_ = ess_compare(gpu_ess_rec, e)
                    if cmp_:
                        gpu_ess_rec["vs_cpu"] = cmp_
                        gpu_ess_rec["z_vs_cpu"] = cmp_["z"]
            c = (calib or {}).get("ratios", {}).get(kind)
            if c and b.get("value"):
                b["reference_equivalent"] = {
                    "value": b["value"] * c["ref_over_port"], "ref_over_port": c["ref_over_port"],
                    "note": "the port's host rate scaled by the reference/port speed ratio measured single-threaded "
                            "in the build container (profiles/cpu_calibration.json, tools/calibrate_cpu_baseline.py)"}
            return b
        out["cpu_baseline"] = baseline("single", out.get("ess"))
        for name, kind in cpu_kinds.items():
            sec[name]["cpu_baseline"] = baseline(kind, sec[name].get("ess"))
    if rank == 0:
        out["secondary"] = sec
        out["detail"] = write_detail(out)
        print(result_line(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
