"""GPU: replayed (hipGraph-captured) training steps — spwgnn_amd/replay.py.

A replayed step must be the step the eager path runs: same dropout masks (the key read from a
device word that spwgnn_step_advance moves on), same Adam step (lr_t from the host-built table),
same batch arrays (refilled in place before each replay). Checked bit for bit:
  * Keras fit with graph=True against graph=False (the same launches issued eagerly), and against
    train_on_batch (host-side key and step, spwgnn_adam) on the same capacity-planned batches;
  * Trainer.replay_body replays against Trainer.step on changing batches.
Reference: the training loop of src/main.py:92-98 (batch 32) and Networks.py:101-102 (Adam, BCE).
"""
import numpy as np
import pytest
import torch

from oracle import model as O
from spwgnn_amd import data as D, engine as E, params as P
from spwgnn_amd.batch import HostPlan, TowerBatch
from spwgnn_amd.keras_api import CompactDataset, PropagationNetwork
from spwgnn_amd.replay import ReplayStep
from spwgnn_amd.trainer import Trainer

pytestmark = pytest.mark.gpu


def _xy(n, seed):
    obj, Rs, Rr, prop, tgt = D.synthetic_batch(n, 6, seed=seed, fully_connected=False)
    return ({"objects": obj, "sender_relations": Rs, "receiver_relations": Rr, "propagation": prop},
            {"target": tgt.reshape(n, 6, 1)})


def test_fit_replayed_equals_eager_bitwise():
    """model.fit with every step a replayed hipGraph == the same fit issued eagerly: per-epoch
    losses/accuracies and the final weights, bit for bit (batch 32 plus a partial last batch: two
    captured geometries), and a second fit call continues from the device counters."""
    x, y = _xy(150, 7)
    res = []
    for graph in (True, False):
        model = PropagationNetwork(seed=0).getModel(6)
        h1 = model.fit(x, y, batch_size=32, epochs=3, validation_split=0.2, verbose=0, graph=graph)
        h2 = model.fit(x, y, batch_size=32, epochs=1, validation_split=0.2, verbose=0, graph=graph, seed=5)
        torch.cuda.synchronize()
        res.append((h1, h2, model.net.flat.detach().cpu().numpy().copy(), model.iterations, model.net._step_seed,
                    model._replays))
    (ha, ha2, wa, ia, ka, ra), (hb, hb2, wb, ib, kb, rb) = res
    assert ha == hb and ha2 == hb2
    assert np.array_equal(wa, wb)
    assert ia == ib == 4 * 4 and ka == kb                    # 120 training towers → 4 steps per epoch
    assert sum(s.replays for s in ra.steps.values()) == 16 - len(ra.steps)   # first call of a geometry is eager
    assert all(s.graph is None for s in rb.steps.values())
    assert ha["loss"][-1] < ha["loss"][0]


def test_fit_steps_equal_train_on_batch():
    """The replayed step's device-side key and Adam step reproduce the host-side path
    (train_on_batch: key from net._step_seed, spwgnn_adam at model.iterations) bit for bit."""
    x, y = _xy(64, 9)
    ma = PropagationNetwork(seed=3).getModel(6)
    ma.fit(x, y, batch_size=32, epochs=1, validation_split=0.0, shuffle=False, verbose=0)
    mb = PropagationNetwork(seed=3).getModel(6)
    ds = CompactDataset(x["objects"], x["sender_relations"], x["receiver_relations"], x["propagation"])
    tgt = y["target"].reshape(64, 6)
    for b0 in (0, 32):
        idx = np.arange(b0, b0 + 32)
        batch = TowerBatch.from_plan(ds.subset_plan(idx, edge_cap=True), "cuda")
        mb.train_on_batch(batch, torch.as_tensor(tgt[idx].reshape(-1), device="cuda"))
    torch.cuda.synchronize()
    assert np.array_equal(ma.net.flat.detach().cpu().numpy(), mb.net.flat.detach().cpu().numpy())
    assert ma.iterations == mb.iterations == 2 and ma.net._step_seed == mb.net._step_seed


def test_trainer_replay_equals_step():
    """Trainer.replay_body (splitmix key mode, x6 math, dropout 0.1) replayed over three different
    batches of one geometry == Trainer.step on the same batches, bit for bit (parameters and both
    Adam moments)."""
    params = O.random_params(12)
    plans, tgts = [], []
    for seed in (1, 2, 3):
        raw = D.synthetic_towers(32, 6, seed=seed)
        obj = (raw / D.RELATION_THRESHOLD).astype(np.float32)
        Rs, Rr = D.relation_matrices(raw, D.RELATION_THRESHOLD)
        e = np.array(O.dense_to_edges(Rs, Rr), np.int64).reshape(-1, 4)
        te = np.bincount(e[:, 0], minlength=32).astype(np.int32)
        plans.append(HostPlan.build(obj.reshape(-1, 3), np.full(32, 6, np.int32), e[:, 0] * 6 + e[:, 2],
                                    e[:, 0] * 6 + e[:, 3], te, edge_cap=30))
        tgts.append(np.random.default_rng(seed).integers(0, 2, 192).astype(np.float32))
    assert len({p.geometry for p in plans}) == 1
    ta = Trainer(P.to_flat(params, device="cuda"), mp_steps=5, dropout=0.1, seed=11, math="x6")
    for p, t in zip(plans, tgts):
        ta.step(TowerBatch.from_plan(p, "cuda"), torch.as_tensor(t, device="cuda"))
    tb = Trainer(P.to_flat(params, device="cuda"), mp_steps=5, dropout=0.1, seed=11, math="x6")
    rs = ReplayStep(plans[0], "cuda", tb.replay_body(plans[0].n_nodes))
    for p, t in zip(plans, tgts):
        tb.replay_step(rs, p, t)
    torch.cuda.synchronize()
    assert rs.replays == 2
    assert torch.equal(ta.params, tb.params) and torch.equal(ta.m, tb.m) and torch.equal(ta.v, tb.v)
    assert int(tb._ctr.step.item()) == 3 and tb.iterations == 3


def _trainer_plans(n):
    plans, tgts = [], []
    for seed in range(1, n + 1):
        raw = D.synthetic_towers(32, 6, seed=seed)
        obj = (raw / D.RELATION_THRESHOLD).astype(np.float32)
        Rs, Rr = D.relation_matrices(raw, D.RELATION_THRESHOLD)
        e = np.array(O.dense_to_edges(Rs, Rr), np.int64).reshape(-1, 4)
        te = np.bincount(e[:, 0], minlength=32).astype(np.int32)
        plans.append(HostPlan.build(obj.reshape(-1, 3), np.full(32, 6, np.int32), e[:, 0] * 6 + e[:, 2],
                                    e[:, 0] * 6 + e[:, 3], te, edge_cap=30))
        tgts.append(np.random.default_rng(seed).integers(0, 2, 192).astype(np.float32))
    return plans, tgts


def test_trainer_replay_reuses_staging_slots():
    """eight different batches of one geometry replayed back to back (graph=True, no host
    synchronisation between steps), so each of the two pinned staging slots is rewritten by the host
    and re-read by the upload (system-coherent loads, device_common.h ld_sys_u4) four times ==
    Trainer.step on the same batches, bit for bit (parameters and both Adam moments)."""
    params = O.random_params(14)
    plans, tgts = _trainer_plans(8)
    assert len({p.geometry for p in plans}) == 1
    ta = Trainer(P.to_flat(params, device="cuda"), mp_steps=3, dropout=0.1, seed=9, math="x6")
    for p, t in zip(plans, tgts):
        ta.step(TowerBatch.from_plan(p, "cuda"), torch.as_tensor(t, device="cuda"))
    tb = Trainer(P.to_flat(params, device="cuda"), mp_steps=3, dropout=0.1, seed=9, math="x6")
    rs = ReplayStep(plans[0], "cuda", tb.replay_body(plans[0].n_nodes))
    for p, t in zip(plans, tgts):
        tb.replay_step(rs, p, t)
    torch.cuda.synchronize()
    assert rs.replays == 7 and rs.static.loads == 8
    assert torch.equal(ta.params, tb.params) and torch.equal(ta.m, tb.m) and torch.equal(ta.v, tb.v)


def test_trainer_replay_mixed_with_step_and_lr_change():
    """replayed steps interleaved with eager Trainer.step calls and an lr change keep
    one step count and the current lr: replay, step, replay (lr halved), step == four eager steps
    with the same lr schedule, bit for bit."""
    params = O.random_params(13)
    plans, tgts = _trainer_plans(4)
    ta = Trainer(P.to_flat(params, device="cuda"), mp_steps=3, dropout=0.1, seed=5, math="x6")
    for i, (p, t) in enumerate(zip(plans, tgts)):
        if i == 2:
            ta.lr = 2.5e-4
        ta.step(TowerBatch.from_plan(p, "cuda"), torch.as_tensor(t, device="cuda"))
    tb = Trainer(P.to_flat(params, device="cuda"), mp_steps=3, dropout=0.1, seed=5, math="x6")
    rs = ReplayStep(plans[0], "cuda", tb.replay_body(plans[0].n_nodes))
    tb.replay_step(rs, plans[0], tgts[0])
    tb.step(TowerBatch.from_plan(plans[1], "cuda"), torch.as_tensor(tgts[1], device="cuda"))
    tb.lr = 2.5e-4
    tb.replay_step(rs, plans[2], tgts[2])
    tb.step(TowerBatch.from_plan(plans[3], "cuda"), torch.as_tensor(tgts[3], device="cuda"))
    torch.cuda.synchronize()
    assert rs.replays == 1 and tb.iterations == 4
    assert torch.equal(ta.params, tb.params) and torch.equal(ta.m, tb.m) and torch.equal(ta.v, tb.v)


def test_fit_lr_change_between_fits():
    """model.lr changed between two fit calls reaches the replayed Adam (the lr table
    is rebuilt in place): equal to the same two fits issued eagerly."""
    x, y = _xy(64, 4)
    res = []
    for graph in (True, False):
        m = PropagationNetwork(seed=2).getModel(6)
        m.fit(x, y, batch_size=32, epochs=1, shuffle=False, verbose=0, graph=graph)
        m.lr = 1e-3
        m.fit(x, y, batch_size=32, epochs=1, shuffle=False, verbose=0, graph=graph)
        torch.cuda.synchronize()
        res.append(m.net.flat.detach().cpu().numpy().copy())
    assert np.array_equal(res[0], res[1])
    # and the lr did change the trajectory
    m = PropagationNetwork(seed=2).getModel(6)
    m.fit(x, y, batch_size=32, epochs=2, shuffle=False, verbose=0, graph=False)
    assert not np.array_equal(res[1], m.net.flat.detach().cpu().numpy())


def test_capacity_plan_equals_compact_plan():
    """a capacity-planned batch (N(N-1) relation slots per tower, fit's plan) gives the
    same logits and weight gradients as the compact plan of the same towers, at the fp32 tolerance
    (the padding blocks are inert; the segment sums' k-block grouping may differ)."""
    from spwgnn_amd import engine as E
    x, y = _xy(48, 21)
    ds = CompactDataset(x["objects"], x["sender_relations"], x["receiver_relations"], x["propagation"])
    idx = np.arange(48)
    flat = P.to_flat(O.random_params(5), device="cuda")
    tgt = torch.as_tensor(y["target"].reshape(-1), device="cuda")
    out = []
    for cap in (True, False):
        b = TowerBatch.from_plan(ds.subset_plan(idx, edge_cap=cap), "cuda")
        run = E.RunConfig(5, training=True, dropout=0.0, math="x6")
        ws = E.Workspace("cuda")
        z = E.forward(flat, b, run, ws)
        _, dz = E.bce(z, tgt, E.BceScratch("cuda"))
        g, _ = E.backward(flat, b, run, ws, dz)
        out.append((z.cpu().numpy().copy(), P.from_flat(g)))
    (za, ga), (zb, gb) = out
    assert np.all(np.abs(za - zb) <= 1e-5 + 1e-5 * np.abs(zb))
    for name, r in gb.items():
        assert np.abs(ga[name] - r).max() <= 1e-5 * np.abs(r).max() + 1e-7, name


def test_copy_in_kernel_moves_pinned_bytes():
    """spwgnn_copy_in (the replayed step's batch upload, one kernel): every byte of a pinned staging
    buffer lands in the device buffer, and misaligned sizes are rejected."""
    from spwgnn_amd.replay import _mapped_device_ptr
    n = 48 * 1024 + 16
    host = torch.empty(n, dtype=torch.uint8, pin_memory=True)
    host.copy_(torch.from_numpy(np.random.default_rng(3).integers(0, 256, n, dtype=np.uint8)))
    dev = torch.zeros(n, dtype=torch.uint8, device="cuda")
    E.copy_in(host, dev, n, src_dev_ptr=_mapped_device_ptr(host))
    torch.cuda.synchronize()
    assert torch.equal(dev.cpu(), host)
    with pytest.raises(Exception):
        E.copy_in(host, dev, n - 8)


@pytest.mark.parametrize("mode", [0, 1])
def test_forward_prologue_equals_separate_launches(mode):
    """spwgnn_run.prologue (a replayed step's batch upload and key/step advance inside the forward's
    first launch) has the effects of spwgnn_copy_in + spwgnn_step_advance issued before the forward:
    the same bytes land, the key and step words move on alike, and the forward that reads the key
    (dropout) gives the same logits bit for bit."""
    from spwgnn_amd.replay import _mapped_device_ptr
    params = P.to_flat(O.random_params(9), device="cuda")
    obj, Rs, Rr, prop, _ = D.synthetic_batch(24, 6, seed=4, fully_connected=False)
    batch = TowerBatch.from_dense(obj, Rs, Rr, prop, device="cuda")
    n = 20 * 1024 + 48
    host = torch.empty(n, dtype=torch.uint8, pin_memory=True)
    host.copy_(torch.from_numpy(np.random.default_rng(5).integers(0, 256, n, dtype=np.uint8)))
    out = []
    for folded in (False, True):
        key = torch.tensor([12345], dtype=torch.int64, device="cuda")
        step = torch.tensor([7], dtype=torch.int32, device="cuda")
        dev = torch.zeros(n, dtype=torch.uint8, device="cuda")
        ws = E.Workspace("cuda")
        run = E.RunConfig(3, training=True, dropout=0.1, seed_dev=key)
        if folded:
            run.prologue = E.Prologue(dst=dev, src_dev_ptr=_mapped_device_ptr(host), nbytes=n, key=key, step=step,
                                      mode=mode, seed=99, rank=1)
        else:
            E.copy_in(host, dev, n, src_dev_ptr=_mapped_device_ptr(host))
            E.step_advance(key, step, mode, 99, 1)
        z = E.forward(params, batch, run, ws)
        torch.cuda.synchronize()
        out.append((dev.cpu(), int(key.item()), int(step.item()), z.cpu()))
    (d0, k0, s0, z0), (d1, k1, s1, z1) = out
    assert torch.equal(d0, host) and torch.equal(d1, host)
    assert (k0, s0) == (k1, s1) and s1 == 8 and k1 != 12345
    assert torch.equal(z0, z1)
    with pytest.raises(Exception):   # misaligned size
        bad = E.RunConfig(3, training=True, prologue=E.Prologue(dst=dev, src_dev_ptr=_mapped_device_ptr(host), nbytes=n - 8))
        E.forward(params, batch, bad, E.Workspace("cuda"))
