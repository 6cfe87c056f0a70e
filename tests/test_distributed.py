"""Multi-process plumbing on CPU (gloo, world_size 2): the sharding helpers and
the per-sweep exchange used by the pulsar-sharded CURN path."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from pulsar_timing_gibbsspec_amd import distributed as D


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, fn, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        q.put((rank, fn(rank, world)))
    finally:
        dist.destroy_process_group()


def run_world(fn, world=2):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, fn, q)) for r in range(world)]
    for p in ps:
        p.start()
    out = dict(q.get(timeout=120) for _ in range(world))
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    return out


def _gather_case(rank, world):
    P, n_f, C = 7, 5, 3
    full = torch.arange(P * 2 * n_f * C, dtype=torch.float64).reshape(P, 2, n_f, C)
    assign = [np.arange(*D.shard_range(P, r, world)) for r in range(world)]
    g = D.PulsarAllGather(assign, (2, n_f, C))
    local = full[assign[rank]]
    out = g(local)
    return bool(torch.equal(out, full)), g.pmax, D.max_over_ranks(float(rank + 1))


def _gather_lpt_case(rank, world):
    w = np.array([5.0, 1, 1, 4, 2, 3, 3])
    assign = D.balance_pulsars(w, world)
    full = torch.randn(len(w), 1, 4, 2, generator=torch.Generator().manual_seed(0), dtype=torch.float64)
    g = D.PulsarAllGather(assign, (1, 4, 2))
    return bool(torch.equal(g(full[assign[rank]]), full))


def test_shard_range_covers_everything():
    for n in (0, 1, 7, 45, 4096):
        for w in (1, 2, 3, 8):
            blocks = [D.shard_range(n, r, w) for r in range(w)]
            assert blocks[0][0] == 0 and blocks[-1][1] == n
            assert all(blocks[i][1] == blocks[i + 1][0] for i in range(w - 1))
            sizes = [b - a for a, b in blocks]
            assert max(sizes) - min(sizes) <= 1


def test_balance_pulsars_by_cost():
    m = np.array([70, 77, 68, 72, 75, 69, 74, 71])
    a = D.balance_pulsars(m ** 3, 3)
    assert sorted(np.concatenate(a).tolist()) == list(range(8))
    loads = [np.sum(m[x] ** 3) for x in a]
    assert max(loads) / min(loads) < 1.5


@pytest.mark.timeout(300)
def test_pulsar_allgather_gloo_world2():
    out = run_world(_gather_case, 2)
    assert all(v[0] for v in out.values())
    assert out[0][1] == 4 and out[0][2] == 2.0 and out[1][2] == 2.0


@pytest.mark.timeout(300)
def test_pulsar_allgather_uneven_lpt_gloo_world2():
    out = run_world(_gather_lpt_case, 2)
    assert all(out.values())


def _allreduce_case(rank, world):
    n_f, C, P = 5, 3, 9
    tau = torch.rand(P, n_f, C, generator=torch.Generator().manual_seed(1), dtype=torch.float64)
    lo, hi = D.shard_range(P, rank, world)
    partial = tau[lo:hi].sum(dim=0)
    out = D.TauSumAllReduce()(partial.clone())
    return out.numpy().tolist(), float(torch.max(torch.abs(out - tau.sum(dim=0))))


def test_tau_sum_allreduce_gloo_world2():
    """The CURN exchange without red noise: per-rank partial tau sums all-reduce to the
    global S_k, identical on every rank."""
    out = run_world(_allreduce_case)
    assert out[0][0] == out[1][0]
    assert out[0][1] < 1e-12



# ------------------------------------------------------------- order-free CURN exchange
def fx_digits(tau, e0):
    """Restatement of k_tau_sum_fx's encoding (csrc/gibbs_grid.hip) with Python integers: the
    three 48-bit digits (as int64 sums) of sum_p floor(tau_p / 2^e0), tau [P, ...] >= 0."""
    from fractions import Fraction
    t = np.asarray(tau, np.float64)
    out = np.zeros((3,) + t.shape[1:], np.int64)
    flat = t.reshape(t.shape[0], -1)
    o = out.reshape(3, -1)
    for j in range(flat.shape[1]):
        d = [0, 0, 0]
        for v in flat[:, j]:
            V = int(Fraction(float(v)) / Fraction(2) ** e0)      # floor (v >= 0)
            for i in range(3):
                d[i] += (V >> (48 * i)) & ((1 << 48) - 1)
        o[:, j] = d
    return out


def fx_value(digits, e0):
    """The exact value the digits stand for, correctly rounded to a double."""
    from fractions import Fraction
    d = np.asarray(digits).reshape(3, -1)
    return np.array([float(Fraction(int(d[0, j]) + (int(d[1, j]) << 48) + (int(d[2, j]) << 96)) * Fraction(2) ** e0)
                     for j in range(d.shape[1])])


def _tau_case():
    g = np.random.default_rng(5)
    P, n_f, C = 45, 6, 4
    # tau over 20 decades (b^2 of weak and strong bins), a few exact zeros
    tau = 10.0 ** g.uniform(-30, -10, (P, n_f, C)) * g.uniform(0.5, 2.0, (P, n_f, C))
    tau[g.random((P, n_f, C)) < 0.02] = 0.0
    return tau, int(np.floor(np.log2(1e-18))) - 64


def _fx_case(rank, world):
    tau, e0 = _tau_case()
    lo, hi = D.shard_range(tau.shape[0], rank, world)
    part = torch.as_tensor(fx_digits(tau[lo:hi], e0))
    out = D.TauSumAllReduce()(part)
    return out.numpy().tolist()


@pytest.mark.timeout(600)
@pytest.mark.parametrize("world", [2, 4, 8])
def test_tau_sum_fixed_point_exchange_is_shard_invariant(world):
    """SURVEY §4 (shard counts 1/2/4/8 give identical chains) for the CURN exchange: the
    per-rank fixed-point digits all-reduced over `world` gloo ranks equal the 1-shard digits
    exactly, on every rank, and stand for the tau sums to double precision."""
    tau, e0 = _tau_case()
    one = fx_digits(tau, e0)
    out = run_world(_fx_case, world)
    for r in range(world):
        assert np.array_equal(np.asarray(out[r], np.int64), one), r
    S = fx_value(one, e0).reshape(tau.shape[1:])
    exact = np.array([[__import__("math").fsum(tau[:, k, c]) for c in range(tau.shape[2])]
                      for k in range(tau.shape[1])])
    assert np.max(np.abs(S - exact) / exact) < 2.3e-16
