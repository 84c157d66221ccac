"""The layer-split pipeline schedule of bench.py (PipelineStage.item: recv -> compute ->
isend, sequences interleaved) on 3 gloo ranks with a numpy stand-in for the stage compute:
every sequence's final output must equal the whole chain applied in order."""
import os
import socket
import sys

import numpy as np
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class FakeSession:
    """h_out = h_in * 2 + (stage id + 1); first stage seeds h from the token."""

    def __init__(self, rank, n_embd):
        self.rank, self.n_embd, self.out = rank, n_embd, []

    def reset(self):
        self.out = []

    def decode_stage(self, tokens=None, h_in=0, n_tokens=None, h_out=0, want_logits=False):
        import ctypes
        n = n_tokens if tokens is None else len(tokens)
        if tokens is not None:
            h = np.repeat(np.asarray(tokens, np.float32)[:, None], self.n_embd, 1)
        else:
            h = np.ctypeslib.as_array((ctypes.c_float * (n * self.n_embd)).from_address(h_in)).reshape(n, self.n_embd).copy()
        y = h * 2 + (self.rank + 1)
        if want_logits:
            self.out.append(y[-1, 0])
            return y
        np.ctypeslib.as_array((ctypes.c_float * (n * self.n_embd)).from_address(h_out))[:] = y.ravel()


def _worker(rank, world, port, q):
    os.environ.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    sys.path.insert(0, ROOT)
    import torch
    import bench
    _, _, _, dist = bench.dist_setup(world)
    st = bench.PipelineStage.__new__(bench.PipelineStage)
    st.dist, st.rank, st.world, st.n_embd, st.torch = dist, rank, world, 4, torch
    st.dev = torch.device("cpu")
    st.host = True
    st.hin = torch.empty((512, 4), dtype=torch.float32)
    st.hout = [torch.empty((512, 4), dtype=torch.float32) for _ in range(2)]
    st.pending, st.flip = [None, None], 0
    st.sessions = [FakeSession(rank, 4) for _ in range(2)]
    rng = np.random.default_rng(0)
    st.tg(rng, 10, 3)
    if st.last:
        q.put([s.out for s in st.sessions])
    dist.barrier()
    dist.destroy_process_group()


def test_pipeline_schedule_three_ranks():
    world, port = 3, _port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    outs = q.get(timeout=120)
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    toks = np.random.default_rng(0).integers(0, 10, size=(2, 3), dtype=np.int32)
    for si in range(2):
        for k in range(3):
            h = float(toks[si, k])
            for r in range(world):
                h = h * 2 + (r + 1)
            assert outs[si][k] == h
