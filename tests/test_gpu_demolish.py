"""Batched simulator-side inference against the reference's one-predict-per-
candidate semantics, restated with the oracle (JengaBuilder.py:236-259, 309-329)."""
import numpy as np
import pytest
import torch

from oracle import model as O
from spwgnn_amd import data as D
from spwgnn_amd import demolish as DM
from spwgnn_amd import engine as E
from spwgnn_amd.batch import TowerBatch
from spwgnn_amd.network import GraphNetwork

pytestmark = pytest.mark.gpu


def _oracle_sum(params, tower_raw, S=5):
    """The reference's per-candidate predict: B=1, relations on /170 coords < 170 (all pairs)."""
    obj = (tower_raw[None] / 170.0)
    Rs, Rr = O.relation_matrices(obj, 170.0)
    z = O.forward_dense(O.to_torch(params), torch.tensor(obj, dtype=torch.float64), torch.tensor(Rs, dtype=torch.float64),
                        torch.tensor(Rr, dtype=torch.float64), torch.zeros(1, obj.shape[1], 100, dtype=torch.float64), S)
    return float(torch.sigmoid(z).sum())


def test_remove_to_demolish_matches_per_candidate_predicts():
    params = O.random_params(31)
    net = GraphNetwork(params=params)
    boxes = D.synthetic_towers(1, 9, seed=12)[0]
    sums, idx = DM.remove_to_demolish(net, boxes)
    ref = np.array([_oracle_sum(params, np.delete(boxes, i, axis=0)) for i in range(len(boxes))])
    assert np.abs(sums - ref).max() <= 1e-5 * np.abs(ref).max()
    assert idx == int(np.argmin(ref))


def test_drop_to_demolish_candidates():
    params = O.random_params(32)
    net = GraphNetwork(params=params)
    base = D.synthetic_towers(1, 6, seed=5)[0]
    rng = np.random.default_rng(0)
    cands = np.repeat(base[None], 40, axis=0)
    cands[:, 0, 0] = rng.uniform(500, 1000, size=40)      # candidate drop positions of object 0
    cands[:, 0, 1] = rng.uniform(400, 600, size=40)
    sums, idx = DM.drop_to_demolish(net, cands)
    ref = np.array([_oracle_sum(params, c) for c in cands])
    assert np.abs(sums - ref).max() <= 1e-5 * np.abs(ref).max()
    assert idx == int(np.argmin(ref))


@pytest.mark.parametrize("mode", sorted(E.READOUT_MODES))
def test_tower_readout_modes_ragged(mode):
    rng = np.random.default_rng(3)
    sizes = rng.integers(4, 17, size=25)
    towers = [D.synthetic_towers(1, int(n), seed=200 + i)[0] for i, n in enumerate(sizes)]
    objs = [(t / 170).astype(np.float32) for t in towers]
    batch = TowerBatch.ragged(objs, relation_threshold=170.0, raw_positions_list=towers, device="cuda")
    z = torch.randn(batch.n_nodes, device="cuda")
    got = E.tower_readout(z, batch, mode).cpu().numpy()
    v = torch.sigmoid(z) if mode.endswith("prob") else z
    parts = torch.split(v.cpu(), [int(n) for n in sizes])
    ref = np.array([(p.mean() if mode.startswith("mean") else p.sum()).item() for p in parts])
    assert np.allclose(got, ref, rtol=1e-6, atol=1e-6)


def test_forward_pooled_is_mean_of_forward():
    params = O.random_params(33)
    net = GraphNetwork(params=params)
    obj, Rs, Rr, prop, _ = D.synthetic_batch(5, 6, seed=9, fully_connected=False)
    pooled = net.forward_pooled(obj, Rs, Rr, prop, mode="mean_prob").cpu().numpy()
    with torch.no_grad():
        probs = net.forward(obj, Rs, Rr, prop).cpu().numpy()[..., 0]
    assert np.allclose(pooled, probs.mean(axis=1), rtol=1e-6, atol=1e-7)
