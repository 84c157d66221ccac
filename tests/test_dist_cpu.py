"""world_size-2 gloo run of bench.py's multi-rank plumbing (dist_setup, barrier,
max/sum over ranks) — the same functions the driver's torchrun launch uses on the
GPU node, exercised on CPU."""
import os
import socket
import sys

import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    sys.path.insert(0, ROOT)
    import bench
    w, r, local, dist = bench.dist_setup(world)
    assert (w, r, local) == (world, rank, rank) and dist.get_backend() == "gloo"
    bench.barrier(dist, local)
    mx = bench.max_over_ranks(dist, 1.5 + rank)
    sm = bench.sum_over_ranks(dist, 128.0)
    q.put((rank, mx, sm))
    dist.destroy_process_group()


def test_two_rank_reductions():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    res = sorted(q.get(timeout=10) for _ in range(world))
    for rank, mx, sm in res:
        assert mx == 2.5          # max of per-rank times
        assert sm == 256.0        # whole-job token count
