"""GPU: BASELINE.json configs 3–5 at their full per-GPU sizes, checked through size-independent
properties: sampled towers against the fp64 oracle, the same towers re-run in a
small batch, gradient linearity over shards, hipGraph replay. All through the C-ABI.

Tolerances as in test_gpu_parity.py: logits |Δ| ≤ 1e-5 + 1e-5·|z|; gradients ≤ 1e-5 of each
tensor's max. These configs are quoted in bf16 by BASELINE.json; the engine computes them in its
fp32-class x6 math, so the fp32 tolerance applies.
"""
import numpy as np
import pytest
import torch

from oracle import model as O
from spwgnn_amd import TowerBatch, data as D, engine as E, params as P

pytestmark = pytest.mark.gpu


def _oracle_logits(params, raw, S, threshold=None):
    obj = (raw / D.RELATION_THRESHOLD).astype(np.float32)
    Rs, Rr = O.relation_matrices(raw, threshold)
    B, N = raw.shape[:2]
    return O.forward_dense(O.to_torch(params), torch.tensor(obj, dtype=torch.float64),
                           torch.tensor(Rs, dtype=torch.float64), torch.tensor(Rr, dtype=torch.float64),
                           torch.zeros(B, N, 100, dtype=torch.float64), S).numpy()


def _close(got, ref):
    return np.all(np.abs(got - ref) <= 1e-5 + 1e-5 * np.abs(ref)), float(np.abs(got - ref).max())


def test_config3_full_size_forward():
    """Config 3: 65,536 fully connected 12-block towers (E = 132), S = 5 — sampled towers equal the
    oracle, and equal a small-batch run of the same towers to rounding."""
    B, N, S = 65536, 12, 5
    params = O.random_params(31)
    raw = D.synthetic_towers(B, N, seed=3)
    obj = (raw / D.RELATION_THRESHOLD).astype(np.float32)
    flat = P.to_flat(params, device="cuda")
    big = TowerBatch.fully_connected(obj, device="cuda")
    z = E.forward(flat, big, E.RunConfig(S), E.Workspace("cuda")).cpu().numpy().reshape(B, N)
    del big
    pick = np.sort(np.random.default_rng(1).choice(B, 16, replace=False))
    ok, err = _close(z[pick], _oracle_logits(params, raw[pick], S))
    assert ok, err
    small = TowerBatch.fully_connected(obj[pick], device="cuda")
    zs = E.forward(flat, small, E.RunConfig(S), E.Workspace("cuda")).cpu().numpy().reshape(len(pick), N)
    assert np.all(np.abs(zs - z[pick]) <= 2e-6 + 2e-6 * np.abs(z[pick])), np.abs(zs - z[pick]).max()


def test_config3_full_size_gradient_linearity():
    """Config 3 training at full size: the weight gradients of the 65,536-tower batch equal the
    size-weighted sum of the gradients of its two halves (BCE is a mean over nodes)."""
    B, N, S = 65536, 12, 5
    params = O.random_params(32)
    raw = D.synthetic_towers(B, N, seed=5)
    obj = (raw / D.RELATION_THRESHOLD).astype(np.float32)
    tgt = np.random.default_rng(2).integers(0, 2, size=(B, N)).astype(np.float32)
    flat = P.to_flat(params, device="cuda")

    def grads(sl):
        batch = TowerBatch.fully_connected(obj[sl], device="cuda")
        ws = E.Workspace("cuda")
        run = E.RunConfig(S, training=True)
        z = E.forward(flat, batch, run, ws)
        _, dz = E.bce(z, torch.as_tensor(tgt[sl], device="cuda").reshape(-1), E.BceScratch("cuda"))
        g, _ = E.backward(flat, batch, run, ws, dz)
        out = P.from_flat(g)
        del batch, ws, z, dz, g
        torch.cuda.empty_cache()
        return out

    full = grads(slice(0, B))
    h1, h2 = grads(slice(0, B // 2)), grads(slice(B // 2, B))
    for k in full:
        comb = (h1[k] + h2[k]) / 2
        assert np.abs(comb - full[k]).max() <= 1e-5 * np.abs(full[k]).max() + 1e-9, k


def test_config4_ragged_shard_sampled():
    """Config 4's per-GPU shard: 131,072 ragged towers of 4–16 blocks (2^20 / 8 GPUs), relations
    thresholded as in training — sampled towers equal the oracle run on each tower alone."""
    B, S = 131072, 5
    params = O.random_params(33)
    rng = np.random.default_rng(7)
    sizes = rng.integers(4, 17, size=B)
    pick = np.sort(rng.choice(B, 12, replace=False))
    towers = {}
    objs, raws = [], []
    for n in range(4, 17):
        idx = np.nonzero(sizes == n)[0]
        raw_n = D.synthetic_towers(len(idx), n, seed=1000 + n)
        for j, t in enumerate(idx):
            towers[t] = raw_n[j]
    for t in range(B):
        raws.append(towers[t])
        objs.append((towers[t] / D.RELATION_THRESHOLD).astype(np.float32))
    rag = TowerBatch.ragged(objs, relation_threshold=D.RELATION_THRESHOLD, raw_positions_list=raws, device="cuda")
    flat = P.to_flat(params, device="cuda")
    z = E.forward(flat, rag, E.RunConfig(S), E.Workspace("cuda")).cpu().numpy()
    off = np.concatenate([[0], np.cumsum(sizes)])
    for t in pick:
        ref = _oracle_logits(params, raws[t][None], S, D.RELATION_THRESHOLD)[0]
        ok, err = _close(z[off[t]:off[t + 1]], ref)
        assert ok, (int(t), err)


def test_config5_full_size_inference_hipgraph():
    """Config 5's per-GPU shard: 8,192 fully connected 32-block towers (E = 992), S = 10, inference
    forward captured into a hipGraph — replay equals eager bitwise; sampled towers equal the oracle."""
    B, N, S = 8192, 32, 10
    params = O.random_params(34)
    raw = D.synthetic_towers(B, N, seed=9)
    obj = (raw / D.RELATION_THRESHOLD).astype(np.float32)
    batch = TowerBatch.fully_connected(obj, device="cuda")
    flat = P.to_flat(params, device="cuda")
    run = E.RunConfig(S)
    ws = E.Workspace("cuda")
    eager = E.forward(flat, batch, run, ws).clone()
    z = torch.empty_like(eager)
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        E.forward(flat, batch, run, ws, logits=z)
    torch.cuda.current_stream().wait_stream(side)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        E.forward(flat, batch, run, ws, logits=z)
    z.zero_()
    g.replay()
    torch.cuda.synchronize()
    assert torch.equal(z, eager)
    got = z.cpu().numpy().reshape(B, N)
    pick = np.sort(np.random.default_rng(3).choice(B, 4, replace=False))
    ok, err = _close(got[pick], _oracle_logits(params, raw[pick], S))
    assert ok, err


# ---------------------------------------------------------------------------------------------
# Config 2 (N = 6, B = 4,096, S = 3, fp32 training) and configs 3–4 in bf16 arithmetic
# (BASELINE.json names bf16 for them; SPWGNN_MATH_BF16 = operands rounded to bf16, one MFMA product,
# fp32 accumulation). Here: full-size properties (linearity, Adam) and the distance of sampled logits
# from the fp64 oracle (|Δ| ≤ 0.05: the bf16 arithmetic's own error, measured ≤ 1.5e-2); the
# arithmetic itself is checked against the bf16-operand emulator in tests/test_gpu_fullsize.py.
# ---------------------------------------------------------------------------------------------
BF16_LOGIT_ATOL = 0.05


def _train_grads(flat, batch, tgt, S, math, dropout=0.0):
    ws = E.Workspace("cuda")
    run = E.RunConfig(S, training=True, math=math, dropout=dropout)
    z = E.forward(flat, batch, run, ws)
    out3, dz = E.bce(z, torch.as_tensor(np.ascontiguousarray(tgt), device="cuda").reshape(-1), E.BceScratch("cuda"))
    g, _ = E.backward(flat, batch, run, ws, dz)
    torch.cuda.synchronize()
    res = (z.cpu().numpy(), float(out3[0]), P.from_flat(g))
    del ws, z, dz, g
    torch.cuda.empty_cache()
    return res


class _Capture:
    """The HIP engine, keeping a host copy of the (accumulated) gradient the Adam step receives."""

    def __init__(self):
        from spwgnn_amd.trainer import HipEngine
        self.e = HipEngine("cuda")
        self.g = None

    def __getattr__(self, k):
        return getattr(self.e, k)

    def adam(self, params, grads, *a):
        self.g = grads.detach().cpu().double().numpy()
        self.e.adam(params, grads, *a)


@pytest.mark.parametrize("math", ["x6", "f32"])
def test_config2_training_parity_small(math):
    """Config 2's shape (6-block towers, thresholded training relations, S = 3): forward, loss and
    every weight gradient of a 16-tower batch equal the fp64 oracle (fp32 tolerance)."""
    params = O.random_params(41)
    obj, Rs, Rr, prop, tgt = D.synthetic_batch(16, 6, seed=21, fully_connected=False)
    batch = TowerBatch.from_dense(obj, Rs, Rr, prop, device="cuda")
    z, loss, g = _train_grads(P.to_flat(params, device="cuda"), batch, tgt, 3, math)
    loss_ref, z_ref, g_ref = O.loss_and_grads(params, obj, Rs, Rr, prop, tgt, 3)
    ok, err = _close(z.reshape(z_ref.shape), z_ref)
    assert ok, err
    assert abs(loss - loss_ref) < 1e-5
    for k, r in g_ref.items():
        assert np.abs(g[k] - r).max() <= 1e-5 * np.abs(r).max() + 1e-7, k


def test_config2_full_batch_training():
    """Config 2 at its full size (4,096 six-block towers, thresholded relations, S = 3) through the
    Trainer (fwd → BCE → bwd → Adam): sampled towers' logits equal the oracle; the batch gradient equals
    the node-weighted sum of its two halves' gradients; the Adam step moves the parameters by the
    Keras-Adam update of that gradient."""
    from spwgnn_amd.trainer import Trainer
    B, N, S = 4096, 6, 3
    params = O.random_params(42)
    obj, Rs, Rr, prop, tgt = D.synthetic_batch(B, N, seed=22, fully_connected=False)
    flat = P.to_flat(params, device="cuda")
    full = TowerBatch.from_dense(obj, Rs, Rr, prop, device="cuda")
    z, _, g = _train_grads(flat, full, tgt, S, "x6")
    pick = np.sort(np.random.default_rng(4).choice(B, 16, replace=False))
    z_ref = O.forward_dense(O.to_torch(params), *(torch.tensor(a[pick], dtype=torch.float64) for a in (obj, Rs, Rr, prop)),
                            S).numpy()
    ok, err = _close(z.reshape(B, N)[pick], z_ref)
    assert ok, err
    halves = [slice(0, B // 2), slice(B // 2, B)]
    hg = [_train_grads(flat, TowerBatch.from_dense(obj[h], Rs[h], Rr[h], prop[h], device="cuda"), tgt[h], S, "x6")[2]
          for h in halves]
    for k in g:
        comb = (hg[0][k] + hg[1][k]) / 2
        assert np.abs(comb - g[k]).max() <= 1e-5 * np.abs(g[k]).max() + 1e-9, k
    cap = _Capture()
    tr = Trainer(flat.clone(), engine=cap, mp_steps=S, dropout=0.0, math="x6")
    tr.step(full, torch.as_tensor(tgt, device="cuda").reshape(-1))
    torch.cuda.synchronize()
    assert np.array_equal(cap.g, P.to_flat(g, device="cpu").double().numpy())   # deterministic
    want = O.KerasAdam(lr=5e-4, beta1=0.9, beta2=0.999, eps=1e-7).step(flat.cpu().double().numpy(), cap.g)
    assert np.abs(tr.params.cpu().double().numpy() - want).max() < 1e-7


def test_config3_bf16_full_size():
    """Config 3 in its BASELINE arithmetic (bf16): 65,536 fully connected 12-block towers, S = 5,
    training forward + backward at full size. Sampled towers' logits are within the bf16 tolerance of
    the fp64 oracle; the full-batch gradients equal the mean of its two halves' gradients (linearity
    of the node-mean BCE; fp32 accumulation, 1e-4 of each tensor's max). A sampled sub-batch's
    gradients against the bf16 emulator: test_gpu_fullsize.test_config3_bf16_full_size_against_emulator."""
    B, N, S = 65536, 12, 5
    params = O.random_params(43)
    raw = D.synthetic_towers(B, N, seed=13)
    obj = (raw / D.RELATION_THRESHOLD).astype(np.float32)
    tgt = np.random.default_rng(6).integers(0, 2, size=(B, N)).astype(np.float32)
    flat = P.to_flat(params, device="cuda")
    z, _, g = _train_grads(flat, TowerBatch.fully_connected(obj, device="cuda"), tgt, S, "bf16")
    z = z.reshape(B, N)
    pick = np.sort(np.random.default_rng(8).choice(B, 16, replace=False))
    z_ref = _oracle_logits(params, raw[pick], S)
    assert np.abs(z[pick] - z_ref).max() <= BF16_LOGIT_ATOL, np.abs(z[pick] - z_ref).max()
    hg = [_train_grads(flat, TowerBatch.fully_connected(obj[h], device="cuda"), tgt[h], S, "bf16")[2]
          for h in (slice(0, B // 2), slice(B // 2, B))]
    for k in g:
        comb = (hg[0][k] + hg[1][k]) / 2
        assert np.abs(comb - g[k]).max() <= 1e-4 * np.abs(g[k]).max() + 1e-9, k


def test_config4_bf16_shard_training():
    """Config 4's per-GPU shard in bf16: 131,072 ragged 4–16-block towers trained as the shard plan
    prescribes (two micro-batches of 65,536 whose node-weighted gradients the Trainer accumulates before
    its one Adam update). Checks: sampled towers' logits within the bf16 tolerance of the oracle;
    the accumulated micro-batch gradient equals the single-batch gradient of the whole shard (linearity
    of the node-mean BCE); the Trainer's update is Keras Adam on that gradient."""
    from spwgnn_amd import shard
    from spwgnn_amd.trainer import Trainer
    B, S = 131072, 5
    params = O.random_params(44)
    pos, sizes, src, dst, te, raws = D.ragged_batch(B, 4, 16, seed=9)
    tgt = np.random.default_rng(10).integers(0, 2, size=int(sizes.sum())).astype(np.float32)
    off = np.concatenate([[0], np.cumsum(sizes)])
    flat = P.to_flat(params, device="cuda")
    whole = TowerBatch.from_edges(pos, sizes, src, dst, te, device="cuda")
    z, _, g = _train_grads(flat, whole, tgt, S, "bf16")
    del whole
    torch.cuda.empty_cache()
    for t in np.sort(np.random.default_rng(11).choice(B, 12, replace=False)):
        ref = _oracle_logits(params, raws[t][None], S, D.RELATION_THRESHOLD)[0]
        assert np.abs(z[off[t]:off[t + 1]] - ref).max() <= BF16_LOGIT_ATOL, int(t)
    mbs = shard.micro_batches(0, B, 65536)
    assert len(mbs) == 2
    batches = [TowerBatch.from_edges(*D.edge_slice(pos, sizes, src, dst, te, a, b), device="cuda") for a, b in mbs]
    tgts = [torch.as_tensor(tgt[off[a]:off[b]], device="cuda") for a, b in mbs]

    cap = _Capture()
    tr = Trainer(flat.clone(), engine=cap, mp_steps=S, dropout=0.0, math="bf16")
    tr.step(batches, tgts, n_global=int(sizes.sum()))
    torch.cuda.synchronize()
    gw = P.to_flat(g, device="cpu").double().numpy()
    assert np.abs(cap.g - gw).max() <= 1e-4 * np.abs(gw).max(), np.abs(cap.g - gw).max()
    want = O.KerasAdam(lr=5e-4, beta1=0.9, beta2=0.999, eps=1e-7).step(flat.cpu().double().numpy(), cap.g)
    assert np.abs(tr.params.cpu().double().numpy() - want).max() < 1e-7
