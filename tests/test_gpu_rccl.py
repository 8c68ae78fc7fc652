"""GPU: the data-parallel step through RCCL on the box's one GPU.

A one-rank `nccl` (= RCCL) process group: its all-reduce is the identity, but the step runs the whole
N > 1 choreography on hardware — the backward's early-gradient event (spwgnn_run.grads_early_event),
the side stream that waits for it, the early piece's async RCCL all-reduce, the late piece's
all-reduce on the step's stream, the waits before Adam (Trainer.reduce_split). Parameters after
three steps equal, bit for bit, a Trainer without the overlap (and without any collective), for one
batch and for micro-batches. (Two RCCL ranks cannot share one GPU; the driver's 8-GPU runs take N > 1.)
"""
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist

from oracle import model as O
from spwgnn_amd import TowerBatch, data as D, params as P
from spwgnn_amd.trainer import Trainer

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.fixture
def rccl_one_rank():
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    try:
        yield
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("micro", [False, True])
def test_rccl_overlapped_step_equals_plain_step(rccl_one_rank, micro):
    assert dist.get_backend() == "nccl"
    params = O.random_params(29)
    pos, sizes, src, dst, te, _ = D.ragged_batch(6000, 4, 16, seed=2)
    n = int(sizes.sum())
    tgt_all = np.random.default_rng(3).integers(0, 2, size=n).astype(np.float32)
    if micro:   # two micro-batches, the last one's backward carries the event
        cut = 3000
        parts = [D.edge_slice(pos, sizes, src, dst, te, 0, cut), D.edge_slice(pos, sizes, src, dst, te, cut, 6000)]
        noff = int(sizes[:cut].sum())
        batches = [TowerBatch.from_edges(*p, device="cuda") for p in parts]
        targets = [torch.tensor(tgt_all[:noff], device="cuda"), torch.tensor(tgt_all[noff:], device="cuda")]
    else:
        batches = TowerBatch.from_edges(pos, sizes, src, dst, te, device="cuda")
        targets = torch.tensor(tgt_all, device="cuda")
    ta = Trainer(P.to_flat(params, device="cuda"), mp_steps=5, dropout=0.1, seed=3, math="x6")
    tb = Trainer(P.to_flat(params, device="cuda"), mp_steps=5, dropout=0.1, seed=3, math="x6", overlap=False)
    assert ta._split() and not tb._split() and ta.world == tb.world == 1
    ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
    for k in range(3):
        if k == 2:
            ta.ar_early_events = ev
        ta.step(batches, targets, n_global=n)
        tb.step(batches, targets, n_global=n)
    torch.cuda.synchronize()
    assert ev[1].query() and ev[0].elapsed_time(ev[1]) >= 0.0
    assert torch.equal(ta.params, tb.params) and torch.equal(ta.m, tb.m) and torch.equal(ta.v, tb.v)
    assert not torch.equal(ta.params, P.to_flat(params, device="cuda"))
