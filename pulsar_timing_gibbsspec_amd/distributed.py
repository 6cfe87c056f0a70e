"""Multi-GPU plumbing: one process per GPU, torch.distributed (RCCL over xGMI).

* Independent units (chains in configs 1-4, pulsars in config 3) are sharded
  with no data-path collective (``shard_range``); each rank offsets its global
  chain ids so Philox streams are disjoint and a sharded run reproduces the
  single-GPU chains bit for bit.
* The common-process (CURN) draw couples pulsars (pta_gibbs.py:191-212).  When
  PULSARS are sharded, the only exchange is one all-gather per sweep of each
  rank's [tau | x_red] slab (2 x P_r x n_f x n_chain doubles), after which every
  rank holds the global, pulsar-ordered inputs of the grid-CDF product and draws
  the common rho identically from the same Philox counter (no broadcast).
"""
from __future__ import annotations

import os

import numpy as np
import torch
import torch.distributed as dist


def env_rank():
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def init_from_env(backend=None):
    """Initialise the default process group from torchrun's environment (127.0.0.1 rendezvous)."""
    rank, world, local = env_rank()
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        kw = {}
        if backend == "nccl":
            torch.cuda.set_device(local)
            kw["device_id"] = torch.device("cuda", local)
        dist.init_process_group(backend, **kw)
    return rank, world, local


def shard_range(n, rank, world):
    """Contiguous balanced block [lo, hi) of n units for this rank."""
    q, r = divmod(int(n), int(world))
    lo = rank * q + min(rank, r)
    return lo, lo + q + (1 if rank < r else 0)


def balance_pulsars(weights, world):
    """Greedy LPT assignment of pulsars to ranks by cost weight (sum of m^3,
    SURVEY.md §8e); each rank's list is returned in increasing (global) order."""
    order = np.argsort(-np.asarray(weights, float), kind="stable")
    load = np.zeros(world)
    out = [[] for _ in range(world)]
    for p in order:
        r = int(np.argmin(load))
        out[r].append(int(p))
        load[r] += weights[p]
    return [np.array(sorted(o), dtype=np.int64) for o in out]


class PulsarAllGather:
    """All-gather of per-pulsar slabs [P_r, ...] into the global [P, ...] array in
    global pulsar order.  Slabs are padded to the largest shard so a single
    all_gather_into_tensor (one RCCL call) moves everything."""

    def __init__(self, assignment, slab_shape, dtype=torch.float64, device="cpu", group=None):
        self.assignment = [np.asarray(a, np.int64) for a in assignment]
        self.world = len(self.assignment)
        self.pmax = max(len(a) for a in self.assignment)
        self.P = sum(len(a) for a in self.assignment)
        self.slab_shape = tuple(slab_shape)
        self.group = group
        self.send = torch.zeros((self.pmax,) + self.slab_shape, dtype=dtype, device=device)
        self.recv = torch.zeros((self.world * self.pmax,) + self.slab_shape, dtype=dtype, device=device)
        # row of the padded receive buffer holding global pulsar p
        src = np.empty(self.P, np.int64)
        for r, a in enumerate(self.assignment):
            src[a] = r * self.pmax + np.arange(len(a))
        self.src = torch.as_tensor(src, device=device)

    def __call__(self, local, out=None):
        n = local.shape[0]
        self.send[:n].copy_(local)
        dist.all_gather_into_tensor(self.recv, self.send, group=self.group)
        res = torch.index_select(self.recv, 0, self.src)
        if out is not None:
            out.copy_(res)
            return out
        return res


class TauSumAllReduce:
    """The CURN exchange without per-pulsar red noise: each rank holds the partial sums
    S_k = sum over its pulsars of tau_p,k as exact fixed-point digits [3, n_f, n_chain] int64
    (gs_tau_sum_fx); one all-reduce SUM (RCCL over xGMI for backend 'nccl') leaves the digits of
    the whole array on every rank.  Integer addition is associative, so the result does not
    depend on the number of shards or on the collective's reduction order: every rank, and the
    unsharded run, rounds the same integers to the same S (gs_fx_to_double) and draws the common
    rho from the same Philox counters (north_star: the only collective of the CURN config).
    A floating-point partial-sum all-reduce would not be reproducible across shard counts."""

    def __init__(self, group=None):
        self.group = group

    def __call__(self, partial):
        dist.all_reduce(partial, op=dist.ReduceOp.SUM, group=self.group)
        return partial


def allreduce_sum(t, group=None):
    """Sum of a small tensor over the ranks of ``group`` (host-side bookkeeping, not the data path:
    the red MH warm-up records, acceptance counts).  gloo reduces on the host, so a device tensor is
    staged through host memory there; RCCL reduces it in place.  Without an initialised process group,
    or in a 1-rank one, the local tensor is the sum (a 1-rank exchange such as ``gather=lambda s: s``
    holds every pulsar) and is returned as it is."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size(group) == 1:
        return t
    if dist.get_backend(group) == "nccl" or t.device.type == "cpu":
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
        return t
    h = t.cpu()
    dist.all_reduce(h, op=dist.ReduceOp.SUM, group=group)
    return h.to(t.device)


def max_over_ranks(value, device="cpu"):
    """Max of a float over ranks (the bench's job time)."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return float(value)
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
