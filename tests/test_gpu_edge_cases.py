"""Edge cases of the batch (GPU, through the C-ABI) against the oracle: towers without any
relation (single boxes, boxes too far apart for the main.py:71-81 threshold), towers of 1–3 boxes
mixed with full-size ones, and a batch in which no tower has an edge at all. Keras handles every
one of these (the Rs/Rr products of Networks.py:32-33,84-88 are then empty or all-zero sums), so the
engine must too: a node without incoming relations sees a = tanh(0) = 0 (Networks.py:88).

Tolerances as in test_gpu_parity.py (logits 1e-5 abs + 1e-5 rel; grads 1e-5 of each tensor's max).
"""
import numpy as np
import pytest
import torch

from oracle import model as O
from spwgnn_amd import TowerBatch, data as D, engine as E, params as P

pytestmark = pytest.mark.gpu
S = 5


def _oracle(params, raw, tgt, threshold):
    """Per-tower oracle loss gradients (mean BCE over the tower's boxes) and logits."""
    obj = (raw / 170.0).astype(np.float32)[None]
    Rs, Rr = O.relation_matrices(raw[None], threshold)
    prop = np.zeros((1, len(raw), 100), np.float32)
    _, z, g = O.loss_and_grads(params, obj, Rs, Rr, prop, tgt[None], S)
    return np.asarray(z).reshape(-1), g


def _run(params, towers, tgts, threshold, math):
    objs = [(t / 170.0).astype(np.float32) for t in towers]
    batch = TowerBatch.ragged(objs, relation_threshold=threshold, raw_positions_list=towers, device="cuda")
    flat = P.to_flat(params, device="cuda")
    ws = E.Workspace("cuda")
    run = E.RunConfig(S, training=True, math=math)
    z = E.forward(flat, batch, run, ws)
    tgt = torch.tensor(np.concatenate(tgts), device="cuda")
    _, dz = E.bce(z, tgt, E.BceScratch("cuda"))
    grads, _ = E.backward(flat, batch, run, ws, dz)
    torch.cuda.synchronize()
    return batch, z.cpu().numpy().reshape(-1), P.from_flat(grads)


def _check(params, towers, threshold, math, seed=0):
    rng = np.random.default_rng(seed)
    tgts = [rng.integers(0, 2, size=len(t)).astype(np.float32) for t in towers]
    batch, z, grads = _run(params, towers, tgts, threshold, math)
    n_tot = sum(len(t) for t in towers)
    ref_g = None
    off = 0
    for t, y in zip(towers, tgts):
        zr, gr = _oracle(params, t, y, threshold)
        got = z[off:off + len(t)]
        assert np.all(np.abs(got - zr) <= 1e-5 + 1e-5 * np.abs(zr)), (len(t), np.abs(got - zr).max())
        w = len(t) / n_tot   # the batch loss is the mean over all boxes of the batch
        ref_g = {k: w * v for k, v in gr.items()} if ref_g is None else {k: ref_g[k] + w * gr[k] for k in ref_g}
        off += len(t)
    for k, ref in ref_g.items():
        err = np.abs(grads[k] - ref).max()
        assert err <= 1e-5 * np.abs(ref).max() + 1e-7, (k, err, np.abs(ref).max())
    return batch, grads


@pytest.mark.parametrize("math", ["x6", "f32"])
def test_no_edge_in_the_whole_batch(math):
    """Single-box towers only: no edge block holds a real edge; the rm/rmp gradients are zero."""
    params = O.random_params(21)
    towers = [D.synthetic_towers(1, 1, seed=40 + i)[0] for i in range(7)]
    batch, grads = _check(params, towers, None, math)
    assert batch.n_edges == 0
    for k in ("rm.0.kernel", "rm.3.bias", "rmp.0.kernel", "rmp.2.bias"):
        assert not np.any(grads[k]), k


@pytest.mark.parametrize("math", ["x6", "f32"])
def test_tiny_towers_mixed_with_full_size(math):
    """1-, 2- and 3-box towers between 6- and 12-box ones, fully connected."""
    params = O.random_params(22)
    sizes = [1, 6, 2, 12, 3, 1, 6, 2]
    towers = [D.synthetic_towers(1, n, seed=60 + i)[0] for i, n in enumerate(sizes)]
    _check(params, towers, None, math, seed=1)


def test_towers_without_relations_under_threshold():
    """Boxes spread ≥ 170 px apart: the thresholded relation set (main.py:71-81) is empty for
    those towers, while the other towers of the batch keep theirs."""
    params = O.random_params(23)
    spread = []
    for i in range(3):
        t = D.synthetic_towers(1, 4, seed=80 + i)[0].copy()
        t[:, 0] = 400.0 + 200.0 * np.arange(4)   # x 200 px apart, same row heights as generated
        t[:, 1] = 110.0 + 200.0 * np.arange(4)
        spread.append(t)
    normal = [D.synthetic_towers(1, 6, seed=90 + i)[0] for i in range(3)]
    towers = [spread[0], normal[0], spread[1], normal[1], spread[2], normal[2]]
    batch, _ = _check(params, towers, 170.0, "x6", seed=2)
    assert batch.n_edges > 0
