"""Pulsar-sharded PTA engine across two PROCESSES on the one GPU (gloo carries the
exchange: distributed.PulsarAllGather for CURN+red, distributed.TauSumAllReduce for
CURN without red noise), against the unsharded engine.  On a node the same code runs
one process per GPU over RCCL (backend 'nccl')."""
import os
import socket

import numpy as np
import pytest

from tests.conftest import gpu_available

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _setup(kind):
    from pulsar_timing_gibbsspec_amd import synthetic
    pta = synthetic.array_pta(kind=kind, n_psr=8, seed=3)
    T, N, R = pta.get_basis(), pta.get_ndiag({}), pta.get_residuals()
    names = pta.param_names
    rind = [i for i, n in enumerate(names) if "rho" in n and "gw" in n]
    hind = np.array([i for i, n in enumerate(names) if "red" in n and "rho" in n])
    red_col = hind.reshape(len(T), -1) if kind == "curn_red" else None
    gwid = [np.arange(t.shape[1] - 60, t.shape[1]) for t in T]
    fixed = [np.full(t.shape[1] - 60, 1e-40) for t in T]
    return T, N, R, names, rind, red_col, gwid, fixed


def _x0_hyper(kind, C, dev):
    """x0 over the priors and, for curn_plred (the reference's default redsample='mh'), the red
    hyper tables (pta_hyper.HyperSpec) of the 8-pulsar array."""
    from pulsar_timing_gibbsspec_amd import synthetic
    from pulsar_timing_gibbsspec_amd.pta_hyper import HyperSpec
    pta = synthetic.array_pta(kind=kind, n_psr=8, seed=3)
    names = pta.param_names
    rng = np.random.default_rng(0)
    x0 = rng.uniform(-9, -4, (C, len(names)))
    if kind != "curn_plred":
        return x0, None
    hidx = np.array([i for i, n in enumerate(names) if "red" in n and ("log10_A" in n or "gamma" in n)])
    sigs = [s for s in (pta.signals[k] for k in pta.signals) if "red" in s.name]
    hyper = HyperSpec(pta, pta.params, sigs, hidx, np.zeros(len(names)), 30, dev)
    x0[:, hyper.hind] = rng.uniform(hyper.hlo_host, hyper.hhi_host, (C, hyper.n_h))
    return x0, hyper


def _worker(rank, world, port, kind, mode, S, out_dir):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from pulsar_timing_gibbsspec_amd import _lib
        from pulsar_timing_gibbsspec_amd.distributed import PulsarAllGather, TauSumAllReduce, shard_range
        from pulsar_timing_gibbsspec_amd.engine import DeviceModel, PTAChains
        T, N, R, names, rind, red_col, gwid, fixed = _setup(kind)
        C = 8
        x0, hyper = _x0_hyper(kind, C, "cuda")
        lo, hi = shard_range(len(T), rank, world)
        ctx = _lib.Context(0, seed=31)
        mdl = DeviceModel(ctx, T[lo:hi], N[lo:hi], R[lo:hi], gwid[lo:hi], fixed[lo:hi])
        assign = [np.arange(*shard_range(len(T), r, world)) for r in range(world)]
        eng = None
        if mode == "sum":
            ex = dict(allreduce=TauSumAllReduce())
        else:
            # the slab: tau and each pulsar's red x values (free spectrum: n_f of them; power law: 2)
            rows = 1 if (red_col is None and hyper is None) else 2
            ex = dict(gather=PulsarAllGather(assign, (rows, 30, C), device="cuda"))
        eng = PTAChains(mdl, len(names), rind, red_col, (1e-18, 1e-8), (1e-20, 1e-8), C, x0,
                        P_global=len(T), psr_lo=lo, curn_mode=mode, hyper=hyper, hyper_warmup=40, **ex)
        assert eng.slab_shape == ex["gather"].slab_shape if mode != "sum" else True
        xr = torch.zeros(S, C, len(names), dtype=torch.float64, device="cuda")
        for i in range(S):
            eng.sweep(x_rec=xr[i])
        np.save(os.path.join(out_dir, f"x{rank}.npy"), xr.cpu().numpy())
        if hyper is not None:
            np.save(os.path.join(out_dir, f"h{rank}.npy"),
                    np.concatenate([[eng.hyper_acl], eng.hyper_acceptance()]))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("kind,mode,world", [("curn", "sum", 2), ("curn", "sum", 4), ("curn_red", "exact", 2),
                                             ("curn_plred", "exact", 2), ("curn_plred", "exact", 4)])
def test_pulsar_sharded_processes(tmp_path, kind, mode, world):
    """world processes on the one GPU, pulsars sharded, against the unsharded engine bit for bit
    (CURN: the fixed-point tau-sum digits all-reduced, order-free for any shard count).
    curn_plred: the red MH block (redsample='mh', the reference's default) pulsar-sharded with no
    new collective -- every rank draws the same step table and applies its own pulsars' steps, the
    (log10_A, gamma) values travel in the [tau | x_red] all-gather; the sweep-0 warm-up's
    aclength_hyper and the acceptance (summed over ranks) equal the unsharded engine's."""
    if not gpu_available():
        pytest.skip("no GPU")
    import torch
    import torch.multiprocessing as mp
    from pulsar_timing_gibbsspec_amd import _lib
    from pulsar_timing_gibbsspec_amd.engine import DeviceModel, PTAChains
    S = 5
    ctxm = mp.get_context("spawn")
    port = _free_port()
    ps = [ctxm.Process(target=_worker, args=(r, world, port, kind, mode, S, str(tmp_path))) for r in range(world)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(timeout=240)
        assert p.exitcode == 0
    T, N, R, names, rind, red_col, gwid, fixed = _setup(kind)
    C = 8
    x0, hyper = _x0_hyper(kind, C, "cuda")
    ref = PTAChains(DeviceModel(_lib.Context(0, seed=31), T, N, R, gwid, fixed), len(names), rind, red_col,
                    (1e-18, 1e-8), (1e-20, 1e-8), C, x0, curn_mode=mode, hyper=hyper, hyper_warmup=40)
    xr = torch.zeros(S, C, len(names), dtype=torch.float64, device="cuda")
    for i in range(S):
        ref.sweep(x_rec=xr[i])
    want = xr.cpu().numpy()
    for r in range(world):
        assert np.array_equal(np.load(tmp_path / f"x{r}.npy"), want), r
    if hyper is not None:
        hw = np.concatenate([[ref.hyper_acl], ref.hyper_acceptance()])
        assert 0 < hw[1:].mean() < 1
        for r in range(world):
            assert np.array_equal(np.load(tmp_path / f"h{r}.npy"), hw), r


def _capture_worker(port, kind, mode, out_dir):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        from pulsar_timing_gibbsspec_amd import _lib
        from pulsar_timing_gibbsspec_amd.distributed import PulsarAllGather, TauSumAllReduce
        from pulsar_timing_gibbsspec_amd.engine import DeviceModel, PTAChains
        T, N, R, names, rind, red_col, gwid, fixed = _setup(kind)
        C = 8
        x0, hyper = _x0_hyper(kind, C, "cuda")
        _, hyper_ref = _x0_hyper(kind, C, "cuda")
        rows = 2 if (red_col is not None or hyper is not None) else 1
        ex = dict(allreduce=TauSumAllReduce()) if mode == "sum" else \
            dict(gather=PulsarAllGather([np.arange(len(T))], (rows, 30, C), device="cuda"))
        # curn_plred: the red MH block (redsample='mh') with the sweep-0 warm-up fixing aclength_hyper
        # eagerly (its allreduce_sum runs before the capture), then the captured sweeps' only
        # collective is the [tau | x_red] all-gather
        hy = dict(hyper=hyper, hyper_warmup=40) if hyper is not None else {}
        hy_ref = dict(hyper=hyper_ref, hyper_warmup=40) if hyper is not None else {}
        # the exchange engine (RCCL collective in every sweep) and the plain one, same seeds
        eng = PTAChains(DeviceModel(_lib.Context(0, seed=31), T, N, R, gwid, fixed), len(names), rind, red_col,
                        (1e-18, 1e-8), (1e-20, 1e-8), C, x0, curn_mode=mode, **hy, **ex)
        ref = PTAChains(DeviceModel(_lib.Context(0, seed=31), T, N, R, gwid, fixed), len(names), rind, red_col,
                        (1e-18, 1e-8), (1e-20, 1e-8), C, x0, curn_mode=mode, **hy_ref)
        assert eng.sharded and not ref.sharded
        eng.sweep()
        rec = eng.capture(4)                      # sweeps 1..4, the all-reduce / all-gather inside
        got = []
        for _ in range(2):
            got.append(eng.replay().clone())
        want = torch.zeros(9, C, len(names), dtype=torch.float64, device="cuda")
        for i in range(9):
            ref.sweep(x_rec=want[i])
        np.save(os.path.join(out_dir, "got.npy"), torch.cat(got).cpu().numpy())
        np.save(os.path.join(out_dir, "want.npy"), want[1:].cpu().numpy())
        assert rec.shape == (4, C, len(names))
        if hyper is not None:
            assert eng.hyper_acl == ref.hyper_acl and eng.hyper.steps_total == ref.hyper.steps_total
            assert torch.equal(eng.hyper.acc_total, ref.hyper.acc_total)
            assert not torch.equal(want[-1][:, hyper.hind], want[0][:, hyper.hind])    # the block moved
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("kind,mode", [("curn", "sum"), ("curn_red", "exact"), ("curn_plred", "exact")])
def test_graph_capture_with_rccl_exchange(tmp_path, kind, mode):
    """PTAChains.capture of sweeps whose exchange is an RCCL collective (1-rank 'nccl' group on the
    one GPU): the collective is a node of the hipGraph, and two replays (8 sweeps) equal 8 eager
    sweeps of the engine without an exchange bit for bit.  curn_plred (the reference's default
    redsample='mh', pta_gibbs.py:689-704): the sweep-0 warm-up (and its aclength all-reduce) runs
    eagerly, the captured sweeps hold the red MH steps and the [tau | x_red] all-gather."""
    if not gpu_available():
        pytest.skip("no GPU")
    import torch.multiprocessing as mp
    p = mp.get_context("spawn").Process(target=_capture_worker, args=(_free_port(), kind, mode, str(tmp_path)))
    p.start()
    p.join(timeout=240)
    assert p.exitcode == 0
    assert np.array_equal(np.load(tmp_path / "got.npy"), np.load(tmp_path / "want.npy"))
