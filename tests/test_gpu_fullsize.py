"""GPU: the headline bench workload checked at full size, and the bf16 arithmetic of BASELINE configs
3–4 against the bf16-operand emulator (oracle/bf16.py) instead of a cosine bound.

Headline (bench.py default): 65,536 fully connected 6-block towers, S = 5, dropout 0.1, x6 math, the
training forward + BCE + backward exactly as a bench step runs it. Checked through
  * linearity: the batch's weight gradients equal the node-weighted sum of its two halves' gradients,
    the halves cut with their batch tower ids so every tower draws the masks it draws in the batch;
  * a sampled 16-tower sub-batch (its towers' batch ids, so the same dropout masks) against the fp64
    oracle run with those masks restated by oracle/dropout.py — fp32 tolerance (logits 1e-5 abs +
    1e-5 rel, gradients 1e-5 of each tensor's max), and the full batch's logits of those towers.
bf16 (SPWGNN_MATH_BF16): logits and every gradient tensor against oracle/bf16.py, which restates the
engine's arithmetic definition (operands rounded to bf16 RNE, fp32 accumulation) on the reference graph:
logits |Δ| ≤ 1e-3 + 1e-3·|z|, gradients ≤ 1e-3 of each tensor's max (vs the bf16 rounding itself,
≈ 4e-3 relative per operand; the fp64 oracle differs from bf16 arithmetic by up to ≈ 0.1 of a tensor's
max on these batches).
"""
import numpy as np
import pytest
import torch

from oracle import bf16 as OB
from oracle import dropout as DR
from oracle import model as O
from spwgnn_amd import TowerBatch, data as D, engine as E, params as P

pytestmark = pytest.mark.gpu

BF16_TOL = 1e-3


def _train(flat, batch, tgt, S, math, dropout=0.0, seed=0):
    ws = E.Workspace("cuda")
    run = E.RunConfig(S, training=True, math=math, dropout=dropout, seed=seed)
    z = E.forward(flat, batch, run, ws)
    out3, dz = E.bce(z, torch.as_tensor(np.ascontiguousarray(tgt), device="cuda").reshape(-1), E.BceScratch("cuda"))
    g, _ = E.backward(flat, batch, run, ws, dz)
    torch.cuda.synchronize()
    res = (z.cpu().numpy(), float(out3[0]), P.from_flat(g))
    del ws, z, dz, g
    torch.cuda.empty_cache()
    return res


def _edges_full(T, N):
    m_idx, j_idx = np.nonzero(~np.eye(N, dtype=bool))
    base = (np.arange(T) * N)[:, None]
    return (base + m_idx[None]).reshape(-1), (base + j_idx[None]).reshape(-1)


def test_headline_training_step_full_size():
    B, N, S, rate, seed = 65536, 6, 5, 0.1, 0x5EED1234ABCD
    params = O.random_params(51)
    raw = D.synthetic_towers_fast(B, N, seed=61)
    obj = (raw / D.RELATION_THRESHOLD).astype(np.float32)
    tgt = np.random.default_rng(62).integers(0, 2, size=(B, N)).astype(np.float32)
    flat = P.to_flat(params, device="cuda")
    z, loss, g = _train(flat, TowerBatch.fully_connected(obj, device="cuda"), tgt, S, "x6", rate, seed)
    z = z.reshape(B, N)
    # linearity over the two halves, each tower keeping its batch id (same masks)
    hz, hg = [], []
    for a, b in ((0, B // 2), (B // 2, B)):
        half = TowerBatch.fully_connected(obj[a:b], device="cuda", tower_ids=np.arange(a, b))
        zh, _, gh = _train(flat, half, tgt[a:b], S, "x6", rate, seed)
        hz.append(zh.reshape(b - a, N))
        hg.append(gh)
    np.testing.assert_allclose(np.concatenate(hz), z, rtol=2e-6, atol=2e-6)
    for k in g:
        comb = (hg[0][k] + hg[1][k]) / 2
        assert np.abs(comb - g[k]).max() <= 1e-5 * np.abs(g[k]).max() + 1e-9, k
    # a sampled sub-batch with the batch's dropout masks, against the fp64 oracle
    pick = np.sort(np.random.default_rng(63).choice(B, 16, replace=False))
    pick[-1] = B - 1                                   # the largest tower id of the batch
    sub = TowerBatch.fully_connected(obj[pick], device="cuda", tower_ids=pick)
    zs, loss_s, gs = _train(flat, sub, tgt[pick], S, "x6", rate, seed)
    zs = zs.reshape(len(pick), N)
    Rs, Rr = O.relation_matrices(raw[pick], None)
    drop_r = DR.relation_mask_towers(seed, rate, pick, N)
    drop_o = DR.object_mask_towers(seed, rate, pick, N)
    assert 0.85 < drop_r.astype(bool).mean() < 0.95
    loss_ref, z_ref, g_ref = O.loss_and_grads(params, obj[pick], Rs, Rr, np.zeros((len(pick), N, 100), np.float32),
                                              tgt[pick], S, drop_r=drop_r, drop_o=drop_o)
    assert np.all(np.abs(zs - z_ref) <= 1e-5 + 1e-5 * np.abs(z_ref)), np.abs(zs - z_ref).max()
    assert np.all(np.abs(z[pick] - z_ref) <= 1e-5 + 1e-5 * np.abs(z_ref)), np.abs(z[pick] - z_ref).max()
    assert abs(loss_s - loss_ref) < 1e-5
    worst = 0.0
    for k, r in g_ref.items():
        err = np.abs(gs[k] - r).max()
        worst = max(worst, err / np.abs(r).max())
        assert err <= 1e-5 * np.abs(r).max() + 1e-7, (k, err / np.abs(r).max())
    print(f"headline sub-batch: worst gradient error {worst:.2e} of the tensor max")


# ------------------------------------------------------------------------------- bf16 emulation
def _bf16_check(got_z, got_g, ref_z, ref_g, what):
    err_z = np.abs(got_z - ref_z)
    assert np.all(err_z <= BF16_TOL + BF16_TOL * np.abs(ref_z)), (what, float(err_z.max()))
    worst = {}
    for k, r in ref_g.items():
        e = np.abs(got_g[k] - r).max() / (np.abs(r).max() + 1e-30)
        worst[k] = e
        assert e <= BF16_TOL, (what, k, e)
    print(f"{what}: logits max|Δ| {err_z.max():.2e}, worst gradient {max(worst.values()):.2e} "
          f"({max(worst, key=worst.get)})")


@pytest.mark.parametrize("N,fully,dropout", [(6, True, 0.0), (9, False, 0.0), (6, False, 0.1), (12, True, 0.1)])
def test_bf16_math_against_bf16_emulator(N, fully, dropout):
    """SPWGNN_MATH_BF16 on a 64-tower batch: logits, loss and every gradient equal the bf16-operand
    emulator (oracle/bf16.py) at 1e-3, with and without dropout (the engine's masks, restated)."""
    params = O.random_params(5)
    obj, Rs, Rr, prop, tgt = D.synthetic_batch(64, N, seed=2, fully_connected=fully)
    batch = TowerBatch.from_dense(obj, Rs, Rr, prop, device="cuda")
    seed = 77
    z, loss, g = _train(P.to_flat(params, device="cuda"), batch, tgt, 5, "bf16", dropout, seed)
    e = np.array(O.dense_to_edges(Rs, Rr), np.int64).reshape(-1, 4)      # (tower, slot, sender, receiver)
    src, dst = e[:, 0] * N + e[:, 2], e[:, 0] * N + e[:, 3]
    dr = do = None
    if dropout:
        full_r = DR.relation_mask_towers(seed, dropout, np.arange(64), N)   # slot order, all E slots
        dr = full_r[e[:, 0], e[:, 1]]
        do = DR.object_mask_towers(seed, dropout, np.arange(64), N).reshape(-1, 100)
    loss_e, z_e, g_e = OB.loss_and_grads(params, obj.reshape(-1, 3), src, dst, prop.reshape(-1, 100),
                                         tgt.reshape(-1), 5, drop_r=dr, drop_o=do)
    _bf16_check(z.reshape(-1), g, z_e, g_e, f"bf16 N={N} fully={fully} dropout={dropout}")
    assert abs(loss - loss_e) <= 1e-4


def test_config3_bf16_full_size_against_emulator():
    """Config 3 in bf16 (65,536 fully connected 12-block towers, S = 5, training): sampled towers'
    logits of the full batch and a sampled 16-tower sub-batch's gradients equal the bf16 emulator
    at 1e-3."""
    B, N, S = 65536, 12, 5
    params = O.random_params(43)
    raw = D.synthetic_towers_fast(B, N, seed=13)
    obj = (raw / D.RELATION_THRESHOLD).astype(np.float32)
    tgt = np.random.default_rng(6).integers(0, 2, size=(B, N)).astype(np.float32)
    flat = P.to_flat(params, device="cuda")
    z, _, _ = _train(flat, TowerBatch.fully_connected(obj, device="cuda"), tgt, S, "bf16")
    z = z.reshape(B, N)
    pick = np.sort(np.random.default_rng(8).choice(B, 16, replace=False))
    zs, _, gs = _train(flat, TowerBatch.fully_connected(obj[pick], device="cuda"), tgt[pick], S, "bf16")
    src, dst = _edges_full(len(pick), N)
    _, z_e, g_e = OB.loss_and_grads(params, obj[pick].reshape(-1, 3), src, dst, np.zeros((len(pick) * N, 100)),
                                    tgt[pick].reshape(-1), S)
    _bf16_check(zs.reshape(-1), gs, z_e, g_e, "config 3 sub-batch")
    assert np.all(np.abs(z[pick].reshape(-1) - z_e) <= BF16_TOL + BF16_TOL * np.abs(z_e))


def test_config4_bf16_shard_against_emulator():
    """Config 4's shard in bf16 (131,072 ragged 4–16-block towers, thresholded relations): sampled
    towers' logits equal the bf16 emulator run on each tower alone, at 1e-3."""
    B, S = 131072, 5
    params = O.random_params(44)
    pos, sizes, src, dst, te, raws = D.ragged_batch(B, 4, 16, seed=9)
    flat = P.to_flat(params, device="cuda")
    z, _, _ = _train(flat, TowerBatch.from_edges(pos, sizes, src, dst, te, device="cuda"),
                     np.zeros(int(sizes.sum()), np.float32), S, "bf16")
    off = np.concatenate([[0], np.cumsum(sizes)])
    eoff = np.concatenate([[0], np.cumsum(te)])
    for t in np.sort(np.random.default_rng(11).choice(B, 12, replace=False)):
        n = int(sizes[t])
        s_t, d_t = src[eoff[t]:eoff[t + 1]] - off[t], dst[eoff[t]:eoff[t + 1]] - off[t]
        ze = OB.forward(O.to_torch(params), torch.tensor(pos[off[t]:off[t + 1]], dtype=torch.float64),
                        torch.as_tensor(s_t, dtype=torch.long), torch.as_tensor(d_t, dtype=torch.long),
                        torch.zeros(n, 100, dtype=torch.float64), S).numpy()
        got = z[off[t]:off[t + 1]]
        assert np.all(np.abs(got - ze) <= BF16_TOL + BF16_TOL * np.abs(ze)), (int(t), np.abs(got - ze).max())
