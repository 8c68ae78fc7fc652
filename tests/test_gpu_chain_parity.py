"""GPU: the wide (large-batch) kernels' gradients against the fp64 oracle — the backward the bench
times, checked directly instead of through linearity.

Batches above the team limit (512 blocks, `spwgnn_team_max_blocks`) run the wide kernels the
headline step runs: the per-block chain encoders and their backwards, the persistent edge kernels,
the dA rebuild (`k_dA_x6`), the warp-specialized W2 gradient (`k_w2grad_ws`) and the batched
stored-operand gradients (`k_wgrad_ws_batch`), reduced by `k_wgrad_reduce_all`. Each case asserts
that it runs them (`spwgnn_fused_path` == 0, block counts above the limit, or the limit set to 0).

Kink-robust by construction. A ReLU's derivative jumps at 0 (Blocks.py:20-28, Networks.py:75-76,
86-90): where an fp32 implementation's pre-activation lands within its rounding of 0 it may take the
other side, and one edge's term then moves across the kink of a summed gradient — DESIGN.md §3w
measured 1.9e-3 of a tensor's max from one such unit at B = 8, N = 12, S = 5, with logits within
1e-6. So the batches are drawn from candidate towers and only towers whose every ReLU pre-activation
(and logit-to-clip distance) sits at least TAU from the kink in the fp64 oracle are kept
(`oracle.model.relu_margins_gather`). TAU = 1e-6 is 5x the largest distance at which §3w saw a flip
(2e-7 of a layer's max, layer maxima ~1) and ~10x the engine's measured logit error.
The criterion then holds without an absolute slack term: per tensor, max |Δ| <= 1e-5 · max |g| and
relative L2 <= 5e-6; logits within the north_star's 1e-5. Measured on MI355X (r6): x6 math worst
max |Δ| 0.5–2.8e-6 of the tensor max and relative L2 0.45–2.3e-6 (largest on rm.0, whose Y is the
end of the encoder backward chain); f32 math 2.3e-7 / 1.9e-7.
"""
import numpy as np
import pytest
import torch

from oracle import dropout as DR
from oracle import model as O
from spwgnn_amd import TowerBatch, data as D, engine as E, params as P

pytestmark = pytest.mark.gpu

TAU = 1e-6
GRAD_MAX_REL = 1e-5
GRAD_L2_REL = 5e-6
TEAM_LIMIT = 512


def _slice(pos, sizes, src, dst, te, keep):
    """Towers `keep` (sorted) of a compact edge-form batch, node ids rebased."""
    off = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
    eoff = np.concatenate([[0], np.cumsum(te)]).astype(np.int64)
    n_rows = np.concatenate([np.arange(off[t], off[t + 1]) for t in keep])
    e_rows = np.concatenate([np.arange(eoff[t], eoff[t + 1]) for t in keep])
    new_off = np.concatenate([[0], np.cumsum(sizes[keep])]).astype(np.int64)
    shift = np.repeat(new_off[:-1] - off[keep], te[keep])
    return (pos[n_rows], sizes[keep].astype(np.int32), (src[e_rows] + shift).astype(np.int32),
            (dst[e_rows] + shift).astype(np.int32), te[keep].astype(np.int32), n_rows, e_rows)


def _kink_free(params, pos, sizes, src, dst, te, S, n_keep, drop_r=None, drop_o=None):
    """Indices (sorted) of the first n_keep candidate towers whose ReLU margins exceed TAU."""
    T = len(sizes)
    marg = O.relu_margins_gather(O.to_torch(params), pos, src, dst, np.zeros((len(pos), 100)),
                                 np.repeat(np.arange(T), sizes), T, S, drop_r=drop_r, drop_o=drop_o)
    ok = np.nonzero(marg > TAU)[0]
    print(f"kink-free towers: {len(ok)} of {T} (TAU {TAU:g})")
    assert len(ok) >= n_keep, (len(ok), n_keep)
    return ok[:n_keep]


def _engine(params, batch, tgt, S, math, dropout=0.0, seed=0):
    flat = P.to_flat(params, device="cuda")
    ws = E.Workspace("cuda")
    run = E.RunConfig(S, training=True, math=math, dropout=dropout, seed=seed)
    assert E.fused_path(batch, run) == 0
    z = E.forward(flat, batch, run, ws)
    out3, dz = E.bce(z, torch.as_tensor(tgt, device="cuda").reshape(-1), E.BceScratch("cuda"))
    g, _ = E.backward(flat, batch, run, ws, dz)
    torch.cuda.synchronize()
    res = z.cpu().numpy().reshape(-1), float(out3[0]), P.from_flat(g)
    del ws, z, dz, g
    torch.cuda.empty_cache()
    return res


def _check(what, got, ref):
    z, loss, g = got
    loss_r, z_r, g_r = ref
    z_r = np.asarray(z_r).reshape(-1)
    dz = np.abs(z - z_r)
    assert np.all(dz <= 1e-5 + 1e-5 * np.abs(z_r)), (what, "logits", dz.max())
    assert abs(loss - loss_r) < 1e-5, (what, loss, loss_r)
    worst_max = worst_l2 = 0.0
    for k, r in g_r.items():
        d = g[k].astype(np.float64) - r
        rel_max = np.abs(d).max() / np.abs(r).max()
        rel_l2 = np.linalg.norm(d) / np.linalg.norm(r)
        worst_max, worst_l2 = max(worst_max, rel_max), max(worst_l2, rel_l2)
        assert rel_max <= GRAD_MAX_REL and rel_l2 <= GRAD_L2_REL, (what, k, rel_max, rel_l2)
    print(f"{what}: logits max|dz| {dz.max():.2e}; gradients worst max|dg|/max|g| {worst_max:.2e}, "
          f"worst rel-L2 {worst_l2:.2e}")


def _fc_edges(T, N):
    m_idx, j_idx = np.nonzero(~np.eye(N, dtype=bool))
    base = (np.arange(T, dtype=np.int64) * N)[:, None]
    return (base + m_idx[None]).reshape(-1).astype(np.int32), (base + j_idx[None]).reshape(-1).astype(np.int32)


@pytest.mark.parametrize("math,dropout", [("x6", 0.0), ("x6", 0.1), ("f32", 0.0)])
def test_headline_shape_wide_kernels_gradients(math, dropout):
    """The headline's towers (fully connected N = 6, S = 5) at 3,000 towers — 2,813 edge blocks and
    563 node blocks, both above the team limit: the exact kernel sequence of the bench step, every
    gradient against the fp64 oracle. With dropout 0.1 the oracle runs the engine's masks
    (oracle/dropout.py), keyed by each kept tower's candidate id."""
    N, S, n_keep, seed = 6, 5, 3000, 0x5EED
    params = O.random_params(51)
    cand = 4800
    raw = D.synthetic_towers_fast(cand, N, seed=71)
    obj = (raw / D.RELATION_THRESHOLD).astype(np.float32)
    src, dst = _fc_edges(cand, N)
    sizes, te = np.full(cand, N, np.int32), np.full(cand, N * (N - 1), np.int32)
    dr = do = None
    if dropout:
        dr = DR.relation_mask_towers(seed, dropout, np.arange(cand), N).reshape(-1, 150)
        do = DR.object_mask_towers(seed, dropout, np.arange(cand), N).reshape(-1, 100)
    keep = _kink_free(params, obj.reshape(-1, 3), sizes, src, dst, te, S, n_keep, dr, do)
    tgt = np.random.default_rng(72).integers(0, 2, size=(n_keep, N)).astype(np.float32)
    batch = TowerBatch.fully_connected(obj[keep], device="cuda", tower_ids=keep)
    assert batch.n_eblocks > TEAM_LIMIT and (batch.n_nodes + 31) // 32 > TEAM_LIMIT and batch.n_wtiles > TEAM_LIMIT
    assert E.team_max_blocks() == TEAM_LIMIT
    got = _engine(params, batch, tgt, S, math, dropout, seed)
    ks, kd = _fc_edges(n_keep, N)
    kdr = None if dr is None else dr.reshape(cand, -1, 150)[keep].reshape(-1, 150)
    kdo = None if do is None else do.reshape(cand, N, 100)[keep].reshape(-1, 100)
    ref = O.loss_and_grads(params, obj[keep].reshape(-1, 3), None, None, np.zeros((n_keep * N, 100)), tgt, S,
                           form="gather", src=ks.astype(np.int64), dst=kd.astype(np.int64), drop_r=kdr, drop_o=kdo)
    _check(f"N=6 fc x{n_keep} {math} dropout {dropout}", got, ref)


def test_config3_tile_shape_wide_kernels_gradients():
    """Config 3's tile shape (fully connected N = 12: 132 edges, 5 edge blocks per tower) at 700 towers
    on the wide kernels (team limit 0 for the call: 700 towers are 263 node blocks), x6 math, S = 5."""
    N, S, n_keep = 12, 5, 700
    params = O.random_params(43)
    cand = 4200
    raw = D.synthetic_towers_fast(cand, N, seed=13)
    obj = (raw / D.RELATION_THRESHOLD).astype(np.float32)
    src, dst = _fc_edges(cand, N)
    keep = _kink_free(params, obj.reshape(-1, 3), np.full(cand, N, np.int32), src, dst,
                      np.full(cand, N * (N - 1), np.int32), S, n_keep)
    tgt = np.random.default_rng(6).integers(0, 2, size=(n_keep, N)).astype(np.float32)
    batch = TowerBatch.fully_connected(obj[keep], device="cuda")
    assert batch.n_eblocks > TEAM_LIMIT
    with E.wide_kernels():
        got = _engine(params, batch, tgt, S, "x6")
    ks, kd = _fc_edges(n_keep, N)
    ref = O.loss_and_grads(params, obj[keep].reshape(-1, 3), None, None, np.zeros((n_keep * N, 100)), tgt, S,
                           form="gather", src=ks.astype(np.int64), dst=kd.astype(np.int64))
    _check(f"N=12 fc x{n_keep} x6 (wide kernels)", got, ref)


@pytest.mark.parametrize("pack", [False, True])
def test_ragged_thresholded_wide_kernels_gradients(pack):
    """Config 4's towers (4–16 boxes, relations thresholded at 170 px, main.py:71-81) at 2,500 kept
    towers, above the team limit on both sides, x6 math, S = 5 — in the input's tower order and packed
    (spwgnn_plan_order, as the bench plans config 4: targets in, logits out through the plan's node
    order)."""
    S, n_keep = 5, 2500
    params = O.random_params(44)
    pos, sizes, src, dst, te, _ = D.ragged_batch(5000, 4, 16, seed=9)
    keep = _kink_free(params, pos, sizes, src, dst, te, S, n_keep)
    kpos, ksz, ksrc, kdst, kte, _, _ = _slice(pos, sizes, src, dst, te, keep)
    n = int(ksz.sum())
    tgt = np.random.default_rng(12).integers(0, 2, size=n).astype(np.float32)
    batch = TowerBatch.from_edges(kpos, ksz, ksrc, kdst, kte, device="cuda", pack=pack)
    assert batch.n_eblocks > TEAM_LIMIT and (n + 31) // 32 > TEAM_LIMIT
    assert len(np.unique(ksz)) == 13 and (kte < ksz * (ksz - 1)).any()
    assert (batch.node_perm is not None) == pack
    z, loss, g = _engine(params, batch, batch.to_plan_order(tgt), S, "x6")
    got = (batch.to_input_order(z), loss, g)
    ref = O.loss_and_grads(params, kpos, None, None, np.zeros((n, 100)), tgt, S, form="gather",
                           src=ksrc.astype(np.int64), dst=kdst.astype(np.int64))
    _check(f"ragged 4-16 thresholded x{n_keep} x6 pack={pack} ({batch.n_eblocks} blocks)", got, ref)


# tools/ht_probe.py's nine shapes: (towers, N, fully connected, S, seed)
PROBE = ((16, 6, True, 5, 1), (16, 6, False, 3, 2), (8, 12, True, 5, 3), (8, 12, True, 1, 3),
         (8, 12, False, 5, 4), (24, 12, True, 5, 5), (6, 16, True, 5, 6), (4, 7, True, 2, 7))


@pytest.mark.parametrize("B,N,fully,S,seed", PROBE)
def test_small_batches_on_wide_kernels(B, N, fully, S, seed):
    """DESIGN.md §3w's probe shapes forced onto the wide kernels (team limit 0): the shape that showed
    1.9e-3 of a tensor max (B = 8, N = 12, S = 5) held to the fp32 criterion once the towers with a
    pre-activation within TAU of a kink are left out. The batch is the probe's towers, kink towers
    replaced by the next kink-free candidates of the same generator."""
    params = O.random_params(40 + seed)
    cand = B * (40 if N >= 16 else 8)   # 16-box towers: ~1 in 20 is kink-free
    obj, Rs, Rr, _, tgt_all = D.synthetic_batch(cand, N, seed=20 + seed, fully_connected=fully)
    e = np.array(O.dense_to_edges(Rs, Rr), np.int64).reshape(-1, 4)
    src, dst = (e[:, 0] * N + e[:, 2]).astype(np.int32), (e[:, 0] * N + e[:, 3]).astype(np.int32)
    te = np.bincount(e[:, 0], minlength=cand).astype(np.int32)
    sizes = np.full(cand, N, np.int32)
    keep = _kink_free(params, obj.reshape(-1, 3), sizes, src, dst, te, S, B)
    print("towers kept:", keep.tolist())
    kpos, ksz, ksrc, kdst, kte, _, _ = _slice(obj.reshape(-1, 3), sizes, src, dst, te, keep)
    tgt = tgt_all[keep].reshape(-1)
    batch = TowerBatch.from_edges(kpos, ksz, ksrc, kdst, kte, device="cuda")
    with E.wide_kernels():
        assert E.team_max_blocks() == 0
        got = _engine(params, batch, tgt, S, "x6")
    assert E.team_max_blocks() == TEAM_LIMIT
    ref = O.loss_and_grads(params, kpos, None, None, np.zeros((len(kpos), 100)), tgt, S, form="gather",
                           src=ksrc.astype(np.int64), dst=kdst.astype(np.int64))
    _check(f"probe B={B} N={N} fully={fully} S={S} (wide kernels)", got, ref)


def test_team_and_wide_kernels_agree_on_one_batch():
    """The same small batch through the team kernels and, with the limit at 0, through the wide ones:
    per-node results (logits, d/d'propagation') bitwise equal — same products in the same order
     — and the weight gradients, whose slab grouping follows the launch shape, equal to
    fp32 rounding."""
    params = O.random_params(9)
    obj, Rs, Rr, _, tgt = D.synthetic_batch(20, 9, seed=4, fully_connected=False)
    prop = (np.random.default_rng(5).standard_normal(obj.shape[:2] + (100,)) * 0.3).astype(np.float32)
    batch = TowerBatch.from_dense(obj, Rs, Rr, prop, device="cuda")
    flat = P.to_flat(params, device="cuda")
    outs = []
    for limit in (TEAM_LIMIT, 0):
        prev = E.team_max_blocks(limit)
        try:
            ws = E.Workspace("cuda")
            run = E.RunConfig(5, training=True, math="x6", dropout=0.1, seed=3)
            assert (E.fused_path(batch, run) != 0) == (limit > 0)
            z = E.forward(flat, batch, run, ws)
            _, dz = E.bce(z, torch.as_tensor(tgt, device="cuda").reshape(-1), E.BceScratch("cuda"))
            g, dp = E.backward(flat, batch, run, ws, dz, want_dprop=True)
            torch.cuda.synchronize()
            outs.append((z.cpu().numpy(), dp.cpu().numpy(), P.from_flat(g)))
        finally:
            E.team_max_blocks(prev)
    np.testing.assert_array_equal(outs[0][0], outs[1][0])
    np.testing.assert_array_equal(outs[0][1], outs[1][1])
    for k, r in outs[0][2].items():
        assert np.abs(outs[1][2][k] - r).max() <= 1e-6 * np.abs(r).max(), k


@pytest.mark.parametrize("n_towers,math", [(3000, "x6"), (3000, "bf16"), (8, "x6")])
def test_backward_with_early_gradient_event_is_bitwise_equal(n_towers, math):
    """spwgnn_run.grads_early_event (the data-parallel overlap): the backward issued as two
    weight-gradient groups — the early range [rmp.1.kernel, end) reduced and the event recorded before
    dA, the relation encoder's backward and the encoder-side gradients — gives the gradients and
    d/d'propagation' of the one-group backward bit for bit (wide kernels at 3,000 towers, the fused
    small-batch backward at 8), and the event completes."""
    params = O.random_params(21)
    obj, Rs, Rr, prop, tgt = D.synthetic_batch(n_towers, 6, seed=3, fully_connected=False)
    batch = TowerBatch.from_dense(obj, Rs, Rr, prop, device="cuda")
    flat = P.to_flat(params, device="cuda")
    out = []
    for split in (False, True):
        ws = E.Workspace("cuda")
        run = E.RunConfig(5, training=True, math=math, dropout=0.1, seed=11)
        z = E.forward(flat, batch, run, ws)
        _, dz = E.bce(z, torch.as_tensor(tgt.reshape(-1), device="cuda"), E.BceScratch("cuda"))
        ev = None
        if split:
            ev = torch.cuda.Event()
            ev.record()
            run.grads_early_event = ev
        g = torch.full_like(flat, float("nan"))
        _, dp = E.backward(flat, batch, run, ws, dz, grads=g, want_dprop=True)
        torch.cuda.synchronize()
        if ev is not None:
            assert ev.query()
        out.append((g, dp))
    assert torch.isfinite(out[1][0]).all()
    assert torch.equal(out[0][0], out[1][0]) and torch.equal(out[0][1], out[1][1])


@pytest.mark.parametrize("math", ["x6", "bf16"])
def test_packed_ragged_plan_equals_input_order(math):
    """The bench's config 4 plan (towers in spwgnn_plan_order's order, 14 % fewer blocks) against the
    same towers in input order: logits back in input order and every gradient agree to rounding — x6
    at the fp32 level on 2,500 kink-free towers; bf16 with dropout 0.1 (each tower keeps its id, so its
    masks) on 5,000 towers, whose operand rounding turns a changed summation grouping into bf16-ulp
    steps, within 1 % relative L2."""
    params = O.random_params(8)
    pos, sizes, src, dst, te, _ = D.ragged_batch(5000, 4, 16, seed=5)
    dropout = 0.1
    if math == "x6":   # fp32-level agreement: kink-free towers (module docstring), dropout off
        dropout = 0.0
        keep = _kink_free(params, pos, sizes, src, dst, te, 5, 2500)
        pos, sizes, src, dst, te, _, _ = _slice(pos, sizes, src, dst, te, keep)
    n = int(sizes.sum())
    tgt = np.random.default_rng(4).integers(0, 2, size=n).astype(np.float32)
    flat = P.to_flat(params, device="cuda")
    res = []
    for pack in (False, True):
        b = TowerBatch.from_edges(pos, sizes, src, dst, te, device="cuda", pack=pack)
        ws = E.Workspace("cuda")
        run = E.RunConfig(5, training=True, math=math, dropout=dropout, seed=99)
        z = E.forward(flat, b, run, ws)
        out3, dz = E.bce(z, torch.as_tensor(b.to_plan_order(tgt), device="cuda"), E.BceScratch("cuda"))
        g, _ = E.backward(flat, b, run, ws, dz)
        torch.cuda.synchronize()
        res.append((b.n_eblocks, b.to_input_order(z.cpu().numpy()), float(out3[0]), P.from_flat(g)))
    (nb0, z0, l0, g0), (nb1, z1, l1, g1) = res
    assert nb1 < 0.9 * nb0
    if math == "x6":
        assert np.abs(z1 - z0).max() <= 2e-6 and abs(l1 - l0) <= 1e-6
        for k in g0:
            assert np.abs(g1[k] - g0[k]).max() <= 4e-6 * np.abs(g0[k]).max(), k
    else:
        assert np.abs(z1 - z0).max() <= 2e-2 and abs(l1 - l0) <= 1e-3
        for k in g0:
            assert np.linalg.norm(g1[k] - g0[k]) <= 1e-2 * np.linalg.norm(g0[k]), k
