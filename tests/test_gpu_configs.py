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
