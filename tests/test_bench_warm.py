"""bench.warm with more than one rank: every rank makes the same number of calls even when the ranks
run at different speeds, so a line whose call holds a collective (the pulsar-sharded sweeps) cannot
hang on mismatched collectives (gloo, 2 ranks on CPU; torch.cuda.synchronize stubbed)."""
import os
import socket
import sys

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _rank(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.synchronize = lambda *a, **k: None
    sys.path.insert(0, ROOT)
    import time

    import bench
    calls = []

    def fn():  # a sweep with a collective; rank 1 is 5x slower
        time.sleep(0.002 if rank == 0 else 0.01)
        t = torch.ones(1)
        dist.all_reduce(t)
        calls.append(int(t.item()))

    n = bench.warm(fn, 2, min_ms=60)
    out[rank] = (n, len(calls), calls.count(world) == len(calls))
    dist.destroy_process_group()


def test_warm_counts_agree_across_ranks():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    out = mp.Manager().dict()
    mp.spawn(_rank, args=(2, port, out), nprocs=2, join=True)
    (n0, c0, ok0), (n1, c1, ok1) = out[0], out[1]
    assert n0 == n1 == c0 == c1 >= 2 and ok0 and ok1
