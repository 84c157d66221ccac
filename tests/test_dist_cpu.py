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


def _split_worker(rank, world, port, q):
    """the N > 1 drop-in headline's control flow (bench.split_headline): gloo only, the
    layer-split child started by rank 0 alone, every rank in the barriers around it"""
    os.environ.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    sys.path.insert(0, ROOT)
    import argparse
    import time
    import bench
    w, r, local, dist = bench.dist_setup(world, backend="gloo")
    assert dist.get_backend() == "gloo"
    calls = []

    def fake_split(args, n):
        calls.append(n)
        time.sleep(0.2)
        tok_s, ms = bench.tg_from_samples([500.0, 400.0], args.tg)
        return {"tg": {"tok_s": tok_s, "ms_per_step": ms, "samples": [500.0, 400.0]}, "pp512_tok_s": 1.0}

    args = argparse.Namespace(steps=2, warmup=1, tg=128, pp=512, model="llama3_8b", no_fa=False)
    line = bench.split_headline(args, w, r, local, dist, run_split=fake_split)
    q.put((rank, calls, line))
    dist.destroy_process_group()


def test_split_headline_two_ranks():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_split_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    res = dict((r, (c, l)) for r, c, l in (q.get(timeout=10) for _ in range(world)))
    assert res[1] == ([], None)                  # rank 1 neither runs the child nor prints
    calls, line = res[0]
    assert calls == [2]
    # K = 2 repetitions of 128 tokens at 500 and 400 tok/s: 256 tokens / (0.256 + 0.32) s
    assert abs(line["value"] - 256 / (128 / 500 + 128 / 400)) < 0.01
    assert abs(line["ms_per_step"] - 1000 * (128 / 500 + 128 / 400) / 2) < 0.01
    assert line["n_gpus"] == 2 and line["scaling"] == "strong" and line["wall_s_all_legs"] >= 0.2
    assert "-sm layer -ts 1,1" in line["config"]["parallelism"]
