"""CPU, gloo: the data-parallel Trainer (tower shards + one all-reduce of the node-weighted flat
gradient + Adam) equals a single-process step on the full batch — equal shards (world 2), unequal
ragged shards of mixed tower sizes (worlds 2 and 4, cut by the cost planner and by hand), and
micro-batch accumulation.

The arithmetic engine here is the oracle (test infrastructure) injected into the product Trainer,
so this covers the N>1 control flow without a GPU; the HIP engine runs the same Trainer on MI355X.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import model as O
from spwgnn_amd import data as D, params as P
from spwgnn_amd.batch import TowerBatch
from spwgnn_amd.shard import micro_batches, plan_shards, shard_weights, tower_cost
from spwgnn_amd.trainer import Trainer


class OracleEngine:
    """fp64 torch-CPU oracle behind the Trainer's engine interface (tests only)."""

    def __init__(self):
        self._layout = P.layout()

    def _params(self, flat):
        f = flat.detach().to(torch.float64)
        return {n: f[o:o + int(np.prod(s))].reshape(s).clone().requires_grad_(True) for n, o, s in self._layout}

    def forward(self, flat, batch, run):
        self.p = self._params(flat)
        pos = batch.pos[:, :3].to(torch.float64)
        src = torch.as_tensor(batch.src, dtype=torch.long)
        dst = torch.as_tensor(batch.dst, dtype=torch.long)
        prop = torch.zeros(batch.n_nodes, 100, dtype=torch.float64)
        self.z = O.forward_gather(self.p, pos, src, dst, prop, run.mp_steps)
        return self.z.detach()

    def loss(self, logits, target):
        loss, g = O.keras_bce_grad(logits.numpy(), target.numpy())
        return torch.tensor([loss, 0.0, float(logits.numel())]), torch.tensor(g)

    def backward(self, flat, batch, run, dlogits):
        self.z.backward(dlogits.to(torch.float64))
        g = torch.zeros_like(flat, dtype=torch.float64)
        for n, o, s in self._layout:
            g[o:o + int(np.prod(s))] = self.p[n].grad.reshape(-1)
        return g

    def adam(self, params, grads, m, v, step, lr, b1, b2, eps, l2, gscale):
        g = gscale * grads + 2 * l2 * params.to(torch.float64)
        m.mul_(b1).add_((1 - b1) * g)
        v.mul_(b2).add_((1 - b2) * g * g)
        lr_t = lr * np.sqrt(1 - b2 ** step) / (1 - b1 ** step)
        params.sub_(lr_t * m / (torch.sqrt(v) + eps))


class OverlapOracleEngine(OracleEngine):
    """The oracle engine with an early-gradient 'event' (a CPU step is synchronous: it is reached when
    backward returns), so the Trainer takes its overlapped two-piece all-reduce (reduce_split)."""
    calls = 0

    def early_event(self):
        OverlapOracleEngine.calls += 1
        return "reached"


def _problem(B=8, N=5):
    obj, Rs, Rr, prop, tgt = D.synthetic_batch(B, N, seed=9, fully_connected=False)
    return obj, Rs, Rr, tgt


def _single(steps):
    obj, Rs, Rr, tgt = _problem()
    batch = TowerBatch.from_dense(obj, Rs, Rr, device="cpu")
    params = P.to_flat(O.random_params(11), dtype=torch.float64)
    tr = Trainer(params, engine=OracleEngine(), mp_steps=3, dropout=0.0)
    tr.m = torch.zeros_like(params)
    tr.v = torch.zeros_like(params)
    for _ in range(steps):
        tr.step(batch, torch.tensor(tgt.reshape(-1), dtype=torch.float64))
    return params.numpy()


def _worker(rank, world, port, steps, out, buckets=1, overlap=False):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    obj, Rs, Rr, tgt = _problem()
    sh = slice(rank * 4, rank * 4 + 4)                      # tower shard of this rank
    batch = TowerBatch.from_dense(obj[sh], Rs[sh], Rr[sh], device="cpu")
    params = P.to_flat(O.random_params(11), dtype=torch.float64)
    eng = OverlapOracleEngine() if overlap else OracleEngine()
    tr = Trainer(params, engine=eng, mp_steps=3, dropout=0.0, buckets=buckets)
    assert tr._split() == overlap
    tr.m = torch.zeros_like(params)
    tr.v = torch.zeros_like(params)
    assert tr.world == world
    if buckets > 1:
        bb = tr.bucket_bounds(params.numel())
        assert len(bb) == buckets and bb[0][0] == 0 and bb[-1][1] == params.numel()
        assert all(x[1] == y[0] and x[1] % 64 == 0 for x, y in zip(bb[:-1], bb[1:]))
    for _ in range(steps):
        tr.step(batch, torch.tensor(tgt[sh].reshape(-1), dtype=torch.float64))
    assert OverlapOracleEngine.calls == (steps if overlap else 0)
    if rank == 0:
        np.save(out, params.numpy())
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("steps", [1, 3])
def test_dp_gloo_world2_equals_full_batch(tmp_path, steps):
    out = str(tmp_path / "p.npy")
    mp.start_processes(_worker, args=(2, _free_port(), steps, out), nprocs=2, join=True, start_method="spawn")
    dp = np.load(out)
    ref = _single(steps)
    assert np.abs(dp - ref).max() < 1e-9
    assert np.abs(ref - P.to_flat(O.random_params(11), dtype=torch.float64).numpy()).max() > 1e-6  # it moved


@pytest.mark.parametrize("buckets", [2, 5])
def test_dp_gloo_world2_split_buckets_equal_full_batch(tmp_path, buckets):
    """the flat gradient all-reduced as `buckets` async pieces (all in flight
    before the first wait) == the single-process full batch to 1e-9 over 3 steps."""
    out = str(tmp_path / "p.npy")
    mp.start_processes(_worker, args=(2, _free_port(), 3, out, buckets), nprocs=2, join=True,
                       start_method="spawn")
    assert np.abs(np.load(out) - _single(3)).max() < 1e-9


def test_dp_gloo_world2_overlapped_allreduce_equals_full_batch(tmp_path):
    """SURVEY §8e / VERDICT r5 item 7: the gradient all-reduced in two pieces — the early range
    [rmp.1.kernel, end) issued first (async), the encoder-side rest after the backward — equals the
    single-process full batch to 1e-9 over 3 steps."""
    out = str(tmp_path / "p.npy")
    mp.start_processes(_worker, args=(2, _free_port(), 3, out, 1, True), nprocs=2, join=True, start_method="spawn")
    assert np.abs(np.load(out) - _single(3)).max() < 1e-9


# ---------------------------------------------------------------- ragged / unequal shards
def _ragged_problem(T=11, seed=5):
    """Towers of 3..8 boxes, thresholded relations (main.py:71-81), Bernoulli labels."""
    rng = np.random.default_rng(seed)
    sizes = rng.integers(3, 9, size=T)
    raws = [D.synthetic_towers(1, int(n), seed=seed * 100 + i)[0] for i, n in enumerate(sizes)]
    objs = [(r / D.RELATION_THRESHOLD).astype(np.float32) for r in raws]
    tgts = [rng.integers(0, 2, size=int(n)).astype(np.float64) for n in sizes]
    return objs, raws, tgts


def _ragged_batch(objs, raws, a, b):
    return TowerBatch.ragged(objs[a:b], relation_threshold=D.RELATION_THRESHOLD, device="cpu",
                             raw_positions_list=raws[a:b])


def _ragged_single(steps, micro=None):
    objs, raws, tgts = _ragged_problem()
    params = P.to_flat(O.random_params(11), dtype=torch.float64)
    tr = Trainer(params, engine=OracleEngine(), mp_steps=2, dropout=0.0)
    tr.m = torch.zeros_like(params)
    tr.v = torch.zeros_like(params)
    T = len(objs)
    cuts = [(0, T)] if micro is None else [(a, min(a + micro, T)) for a in range(0, T, micro)]
    bs = [_ragged_batch(objs, raws, a, b) for a, b in cuts]
    ts = [torch.tensor(np.concatenate(tgts[a:b])) for a, b in cuts]
    for _ in range(steps):
        tr.step(bs if micro else bs[0], ts if micro else ts[0])
    return params.numpy()


def _ragged_worker(rank, world, port, steps, out, mode):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    objs, raws, tgts = _ragged_problem()
    T = len(objs)
    tn = np.array([len(o) for o in objs])
    if mode == "planned":
        full = _ragged_batch(objs, raws, 0, T)
        ranges = plan_shards(full.tower_nodes, full.tower_edges, world, mp_steps=2)
        n_global = int(tn.sum())
    else:                                   # hand-cut, deliberately unequal; n_global via all-reduce
        cuts = [0, 3, T] if world == 2 else [0, 1, 4, 9, T]
        ranges = [(cuts[r], cuts[r + 1]) for r in range(world)]
        n_global = None
    a, b = ranges[rank]
    params = P.to_flat(O.random_params(11), dtype=torch.float64)
    tr = Trainer(params, engine=OverlapOracleEngine() if mode == "micro_overlap" else OracleEngine(), mp_steps=2,
                 dropout=0.0)
    tr.m = torch.zeros_like(params)
    tr.v = torch.zeros_like(params)
    if mode.startswith("micro"):                     # this rank's shard as micro-batches of ≤ 2 towers
        mbs = micro_batches(a, b, 2)
        bs = [_ragged_batch(objs, raws, x, y) for x, y in mbs]
        ts = [torch.tensor(np.concatenate(tgts[x:y])) for x, y in mbs]
    else:
        bs = _ragged_batch(objs, raws, a, b)
        ts = torch.tensor(np.concatenate(tgts[a:b]))
    for _ in range(steps):
        tr.step(bs, ts, n_global=n_global)
    if rank == 0:
        np.save(out, params.numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,mode", [(2, "planned"), (2, "unequal"), (4, "planned"), (4, "unequal"),
                                        (2, "micro"), (2, "micro_overlap")])
def test_dp_gloo_ragged_unequal_shards_equal_full_batch(tmp_path, world, mode):
    out = str(tmp_path / "p.npy")
    mp.start_processes(_ragged_worker, args=(world, _free_port(), 2, out, mode), nprocs=world, join=True,
                       start_method="spawn")
    dp = np.load(out)
    ref = _ragged_single(2)
    assert np.abs(dp - ref).max() < 1e-9


def test_micro_batch_accumulation_equals_full_batch():
    """Single process: micro-batches of 3 towers accumulate to the full-batch step."""
    assert np.abs(_ragged_single(2, micro=3) - _ragged_single(2)).max() < 1e-9


def test_plan_shards_balances_cost():
    rng = np.random.default_rng(0)
    n = rng.integers(4, 17, size=5000)
    e = n * (n - 1)
    cost = tower_cost(n, e)
    for world in (1, 2, 3, 4, 8):
        ranges = plan_shards(n, e, world)
        assert ranges[0][0] == 0 and ranges[-1][1] == len(n)
        assert all(ranges[i][1] == ranges[i + 1][0] for i in range(world - 1))
        per = np.array([cost[a:b].sum() for a, b in ranges])
        assert np.abs(per - cost.sum() / world).max() <= cost.max()
        w = shard_weights(n, ranges)
        assert abs(w.sum() - 1.0) < 1e-12
    # balanced by cost, not by tower count: big towers first → the first shard holds fewer towers
    n2 = np.array([16] * 100 + [4] * 100)
    r = plan_shards(n2, n2 * (n2 - 1), 2)
    assert r[0][1] < 100


# ---------------------------------------------------------------- the bench's own DP workload path
def _bench_cfg():
    import bench
    # BASELINE config 4 (ragged 4-16, thresholded, S=5, micro-batched) scaled to 5 towers per rank,
    # micro-batches of 2: the same make_workload → plan_shards → micro_batches → Trainer path
    cfg = dict(bench.CONFIGS[4], towers=5, micro=2, S=2)
    return bench, cfg


def _bench_worker(rank, world, port, steps, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    bench, cfg = _bench_cfg()
    batches, targets, n_global = bench.make_workload(cfg, rank, "cpu", world)
    params = P.to_flat(O.random_params(11), dtype=torch.float64)
    tr = Trainer(params, engine=OracleEngine(), mp_steps=cfg["S"], dropout=0.0)
    tr.m = torch.zeros_like(params)
    tr.v = torch.zeros_like(params)
    for _ in range(steps):
        out3 = tr.step([b for b in batches], [t.double() for t in targets], n_global)
    assert abs(float(out3[2]) - sum(b.n_nodes for b in batches)) < 1e-9
    np.save(out + f".{rank}.npy", params.numpy())
    dist.barrier()
    dist.destroy_process_group()


def test_bench_workload_dp_gloo_world2_equals_single_process(tmp_path):
    """bench.make_workload at world 2: both ranks build the same global ragged batch (one seed), cut it
    with shard.plan_shards and take n_global from the plan (no node-count all-reduce); the DP step over
    the two shards' micro-batches equals the single-process step on the whole global batch."""
    out = str(tmp_path / "p")
    mp.start_processes(_bench_worker, args=(2, _free_port(), 2, out), nprocs=2, join=True, start_method="spawn")
    bench, cfg = _bench_cfg()
    single = dict(cfg, towers=10)                 # the same 10-tower global batch in one process
    batches, targets, n_global = bench.make_workload(single, 0, "cpu", 1)
    assert n_global == sum(b.n_nodes for b in batches)
    params = P.to_flat(O.random_params(11), dtype=torch.float64)
    tr = Trainer(params, engine=OracleEngine(), mp_steps=cfg["S"], dropout=0.0)
    tr.m = torch.zeros_like(params)
    tr.v = torch.zeros_like(params)
    for _ in range(2):
        tr.step(batches, [t.double() for t in targets], n_global)
    for r in range(2):
        assert np.abs(np.load(out + f".{r}.npy") - params.numpy()).max() < 1e-9
    # and the plan really split the global batch: both ranks hold towers
    w0 = bench.make_workload(cfg, 0, "cpu", 2)
    w1 = bench.make_workload(cfg, 1, "cpu", 2)
    assert sum(b.n_towers for b in w0[0]) + sum(b.n_towers for b in w1[0]) == 10
    assert min(sum(b.n_towers for b in w[0]) for w in (w0, w1)) >= 1 and w0[2] == w1[2] == n_global


def test_dropout_key_fields_do_not_collide():
    """Trainer dropout keys: distinct for every (step, rank, micro) combination, including ranks and
    micro indices past the field widths of the old packed key (4099 ranks, 257 micro-batches)."""
    from spwgnn_amd.trainer import dropout_key
    keys = {dropout_key(7, it, rank, micro) for it in (0, 1) for rank in (0, 1, 4098, 4099, 4100)
            for micro in (0, 1, 256, 257, 258)}
    assert len(keys) == 2 * 5 * 5
    assert dropout_key(7, 0, 0, 257) != dropout_key(7, 0, 1, 0)
