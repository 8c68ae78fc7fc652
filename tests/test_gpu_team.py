"""GPU: the small-batch team kernels (spwgnn_amd/csrc/kernels_team.hip) against the one-wave-per-block
kernels on the same towers.

A batch above kTeamMaxBlocks (512 edge and node blocks) runs every chain kernel one wave per block; a
sub-batch of its first towers, built with their batch tower ids (so every tower draws the dropout
masks it draws in the big batch), runs the team kernels. A team kernel gives each output tile the
same products in the same order, so the per-node results — logits, and d/d'propagation' from the same
dlogits rows — must be bitwise equal. (The weight gradients are sums over the batch and differ.)
The team path's parity with the fp64 oracle is covered by every small-batch test of test_gpu_parity.py.
"""
import numpy as np
import pytest
import torch

from spwgnn_amd import TowerBatch, data as D, engine as E, params as P
from oracle import model as O

pytestmark = pytest.mark.gpu


def _run(flat, batch, S, math, rate, seed, dz_rows):
    ws = E.Workspace("cuda")
    run = E.RunConfig(S, training=True, math=math, dropout=rate, seed=seed)
    z = E.forward(flat, batch, run, ws)
    dz = torch.as_tensor(dz_rows[: batch.n_nodes], device="cuda")
    _, dprop = E.backward(flat, batch, run, ws, dz, want_dprop=True)
    torch.cuda.synchronize()
    return z.cpu().numpy(), dprop.cpu().numpy()


@pytest.mark.parametrize("math", ["x6", "bf16"])
def test_team_kernels_bitwise_equal_wide_kernels(math):
    B, N, S, rate, seed = 3000, 6, 3, 0.1, 0x7EA
    raw = D.synthetic_towers_fast(B, N, seed=71)
    obj = (raw / D.RELATION_THRESHOLD).astype(np.float32)
    prop = (np.random.default_rng(72).standard_normal((B, N, 100)) * 0.3).astype(np.float32)
    dz = (np.random.default_rng(73).standard_normal(B * N) * 1e-2).astype(np.float32)
    flat = P.to_flat(O.random_params(74), device="cuda")
    big = TowerBatch.fully_connected(obj, prop, device="cuda", nw_max=16)   # same wave-tiles in both
    assert big.n_eblocks > 512 and (big.n_nodes + 31) // 32 > 512   # every kernel one wave per block
    zb, pb = _run(flat, big, S, math, rate, seed, dz)
    k = 40
    sub = TowerBatch.fully_connected(obj[:k], prop[:k], device="cuda", nw_max=16, tower_ids=np.arange(k))
    assert sub.n_eblocks <= 512   # every chain kernel in team mode
    zs, ps = _run(flat, sub, S, math, rate, seed, dz)
    n = k * N
    np.testing.assert_array_equal(zs, zb[:n])
    np.testing.assert_array_equal(ps, pb[:n])
    assert np.abs(ps).max() > 0
