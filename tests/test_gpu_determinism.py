"""GPU: run-to-run determinism with a poisoned workspace. One training forward + backward on a fresh
workspace, then again on a workspace whose every byte is 0xFF (NaN as fp32) and a NaN-filled gradient
buffer: logits and every gradient must be bitwise equal. A kernel that reads workspace it did not
write, or an accumulator it did not initialise, fails here whatever the values happen to be (the wide
edge forward once lost its accumulator zeroing: 3 % of a thresholded batch's logits moved by up to
2.6e-2 between two runs, tools/determinism.py). Wide and team kernels, all three maths."""
import numpy as np
import pytest
import torch

from oracle import model as O
from spwgnn_amd import TowerBatch, data as D, engine as E, params as P

pytestmark = pytest.mark.gpu


def _batch(kind, B, seed):
    if kind == "ragged":
        pos, sizes, src, dst, te, _ = D.ragged_batch(B, 4, 16, seed=seed, threshold=D.RELATION_THRESHOLD)
        return TowerBatch.from_edges(pos, sizes, src, dst, te, device="cuda", pack=True)
    N, fully = kind
    obj, Rs, Rr, prop, _ = D.synthetic_batch(B, N, seed=seed, fully_connected=fully)
    return TowerBatch.from_dense(obj, Rs, Rr, prop, device="cuda")


def _step(flat, batch, run, ws, tgt):
    grads = torch.full_like(flat, float("nan"))
    z = E.forward(flat, batch, run, ws)
    _, dz = E.bce(z, tgt, E.BceScratch("cuda"))
    g, _ = E.backward(flat, batch, run, ws, dz, grads=grads)
    torch.cuda.synchronize()
    return z.clone(), g.clone()


@pytest.mark.parametrize("kind,B,math", [
    ((6, False), 3000, "x6"),     # wide kernels, thresholded (config 2's shape)
    ((6, True), 3000, "x6"),      # wide, the headline's shape
    ((12, True), 700, "x6"),
    ((12, True), 700, "bf16"),    # bf16 storage of A, U, V and the node arrays
    ("ragged", 2500, "bf16"),     # config 4's shape, packed plan
    ((6, False), 40, "x6"),       # the fused small-batch loops
    ((6, False), 40, "bf16"),
    ((6, False), 600, "f32"),
    ((20, True), 300, "x6"),      # 17–32-node wave-tiles (W8 edge forward, fp32 storage)
    ((20, True), 300, "bf16"),    # … in bf16 math: A, U, V rounded into fp32 storage
])
def test_repeat_on_poisoned_workspace_is_bitwise(kind, B, math):
    batch = _batch(kind, B, seed=21)
    flat = P.to_flat(O.random_params(3), device="cuda")
    run = E.RunConfig(5, training=True, math=math, dropout=0.1, seed=9)
    tgt = torch.tensor(np.random.default_rng(1).integers(0, 2, batch.n_nodes).astype(np.float32), device="cuda")
    z0, g0 = _step(flat, batch, run, E.Workspace("cuda"), tgt)
    ws = E.Workspace("cuda")
    ws.get(E.workspace_bytes(batch, run)).fill_(0xFF)
    z1, g1 = _step(flat, batch, run, ws, tgt)
    assert torch.isfinite(z0).all() and torch.isfinite(g0).all()
    bad_z = int((z0 != z1).sum())
    bad_g = [name for name, o, shape in P.layout()
             if not torch.equal(g0[o:o + int(np.prod(shape))], g1[o:o + int(np.prod(shape))])]
    assert bad_z == 0 and not bad_g, f"logits differing {bad_z}, gradients differing {bad_g}"


@pytest.mark.parametrize("N,B,math,recv", [(32, 300, "x6", True), (32, 300, "x6", False), (12, 3000, "x6", False),
                                            (12, 3000, "bf16", False), (6, 40, "x6", False)])
def test_inference_repeat_on_poisoned_workspace_is_bitwise(N, B, math, recv):
    """The inference forward (two-slot P/U/V/H2s rotation, receiver-block plans of config 5)."""
    obj, Rs, Rr, prop, _ = D.synthetic_batch(B, N, seed=22, fully_connected=True)
    if N > 16:   # receiver-block plan (spwgnn_plan_fill_recv, as config 5 plans its towers) or not
        m_idx, j_idx = np.nonzero(~np.eye(N, dtype=bool))
        src = (np.arange(B)[:, None] * N + m_idx[None]).reshape(-1).astype(np.int32)
        dst = (np.arange(B)[:, None] * N + j_idx[None]).reshape(-1).astype(np.int32)
        batch = TowerBatch.from_edges(obj.reshape(B * N, 3), np.full(B, N, np.int32), src, dst,
                                      np.full(B, N * (N - 1), np.int32), device="cuda", recv_blocks=recv)
    else:
        batch = TowerBatch.from_dense(obj, Rs, Rr, prop, device="cuda")
    flat = P.to_flat(O.random_params(4), device="cuda")
    run = E.RunConfig(10 if N == 32 else 5, training=False, math=math)
    z0 = E.forward(flat, batch, run, E.Workspace("cuda")).clone()
    ws = E.Workspace("cuda")
    ws.get(E.workspace_bytes(batch, run)).fill_(0xFF)
    z1 = E.forward(flat, batch, run, ws).clone()
    torch.cuda.synchronize()
    assert torch.isfinite(z0).all()
    assert torch.equal(z0, z1), f"{int((z0 != z1).sum())} logits differ"
