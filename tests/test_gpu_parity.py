"""HIP path vs the CPU oracle (fp64) — the parity gate. Runs on an MI355X only (-m gpu).

Tolerances (fp32 kernels vs fp64 oracle): logits |Δ| <= 1e-5 + 1e-5·|z| (north_star: "outputs match
the CPU reference logits within 1e-5 fp32"); gradients |Δ| <= 1e-5·max|g| + 1e-7 per tensor.
"""
import numpy as np
import pytest
import torch

from oracle import model as O
from spwgnn_amd import TowerBatch, data as D, engine as E, params as P

pytestmark = pytest.mark.gpu

LOGIT_ATOL = 1e-5
LOGIT_RTOL = 1e-5


def _oracle_logits(params, obj, Rs, Rr, prop, S):
    tp = O.to_torch(params)
    z = O.forward_dense(tp, torch.tensor(obj, dtype=torch.float64), torch.tensor(Rs, dtype=torch.float64),
                        torch.tensor(Rr, dtype=torch.float64), torch.tensor(prop, dtype=torch.float64), S)
    return z.numpy()


def _gpu_forward(params, batch, S, training=False, math="x6"):
    flat = P.to_flat(params, device="cuda")
    ws = E.Workspace("cuda")
    z = E.forward(flat, batch, E.RunConfig(S, training=training, math=math), ws)
    torch.cuda.synchronize()
    return flat, ws, z


@pytest.mark.parametrize("math", ["x6", "f32"])
@pytest.mark.parametrize("S", [1, 3, 5])
@pytest.mark.parametrize("fully", [True, False])
def test_forward_parity_small(S, fully, math):
    params = O.random_params(seed=3)
    obj, Rs, Rr, prop, _ = D.synthetic_batch(8, 6, seed=11, fully_connected=fully)
    batch = TowerBatch.from_dense(obj, Rs, Rr, prop, device="cuda")
    _, _, z = _gpu_forward(params, batch, S, math=math)
    ref = _oracle_logits(params, obj, Rs, Rr, prop, S)
    got = z.cpu().numpy().reshape(ref.shape)
    err = np.abs(got - ref)
    print(f"S={S} fully={fully} max|dz|={err.max():.3e} max|z|={np.abs(ref).max():.3f}")
    assert np.all(err <= LOGIT_ATOL + LOGIT_RTOL * np.abs(ref))


@pytest.mark.parametrize("N", [3, 5, 9, 12, 16])
def test_forward_parity_sizes(N):
    params = O.random_params(seed=5)
    obj, Rs, Rr, prop, _ = D.synthetic_batch(5, N, seed=N, fully_connected=False)
    rng = np.random.default_rng(N)
    prop = rng.normal(0, 0.3, size=prop.shape).astype(np.float32)   # non-zero propagation input
    batch = TowerBatch.from_dense(obj, Rs, Rr, prop, device="cuda")
    _, _, z = _gpu_forward(params, batch, 5)
    ref = _oracle_logits(params, obj, Rs, Rr, prop, 5)
    got = z.cpu().numpy().reshape(ref.shape)
    assert np.all(np.abs(got - ref) <= LOGIT_ATOL + LOGIT_RTOL * np.abs(ref)), np.abs(got - ref).max()


# (towers, nodes, nw_max): nw_max <= 16 runs the backward segment sums as a one-hot matrix product,
# larger wave-tiles walk the block csr through LDS — both paths, single- and multi-tower tiles.
@pytest.mark.parametrize("math", ["x6", "f32"])
@pytest.mark.parametrize("T,N,nw", [(6, 6, None), (6, 6, 6), (5, 16, None), (7, 5, 32), (3, 20, None), (2, 32, None)])
def test_backward_parity_small(T, N, nw, math):
    params = O.random_params(seed=7)
    obj, Rs, Rr, prop, tgt = D.synthetic_batch(T, N, seed=2, fully_connected=False)
    S = 5
    loss_ref, z_ref, g_ref = O.loss_and_grads(params, obj, Rs, Rr, prop, tgt, S)
    batch = TowerBatch.from_dense(obj, Rs, Rr, prop, device="cuda", nw_max=nw)
    flat, ws, z = _gpu_forward(params, batch, S, training=True, math=math)
    scratch = E.BceScratch("cuda")
    out3, dz = E.bce(z, torch.tensor(tgt, device="cuda").reshape(-1), scratch)
    grads, _ = E.backward(flat, batch, E.RunConfig(S, training=True, math=math), ws, dz)
    torch.cuda.synchronize()
    assert abs(float(out3[0]) - loss_ref) < 1e-5
    got = P.from_flat(grads)
    worst = 0.0
    for name, ref in g_ref.items():
        scale = np.abs(ref).max()
        err = np.abs(got[name] - ref).max()
        worst = max(worst, err / (scale + 1e-30))
        print(f"{name:14s} max|g|={scale:.3e} max|dg|={err:.3e}")
        assert err <= 1e-5 * scale + 1e-7, name
    print("worst relative", worst)


@pytest.mark.parametrize("math", ["x6", "f32"])
@pytest.mark.parametrize("S", [1, 2, 10])
def test_backward_parity_step_counts(S, math):
    """Other propagation-step counts than the reference's 5: S = 1 (no step reuses c_o·Wo1c, the
    Σ_s do1_s of the c_o gradients is one step, the backward writes dA once and never accumulates),
    S = 2 and S = 10 (config 5's step count)."""
    params = O.random_params(seed=17)
    obj, Rs, Rr, prop, tgt = D.synthetic_batch(5, 7, seed=9, fully_connected=False)
    prop = np.random.default_rng(S).normal(0, 0.3, size=prop.shape).astype(np.float32)
    loss_ref, z_ref, g_ref = O.loss_and_grads(params, obj, Rs, Rr, prop, tgt, S)
    batch = TowerBatch.from_dense(obj, Rs, Rr, prop, device="cuda")
    flat, ws, z = _gpu_forward(params, batch, S, training=True, math=math)
    out3, dz = E.bce(z, torch.tensor(tgt, device="cuda").reshape(-1), E.BceScratch("cuda"))
    grads, _ = E.backward(flat, batch, E.RunConfig(S, training=True, math=math), ws, dz)
    torch.cuda.synchronize()
    ref = np.asarray(z_ref).reshape(-1)
    assert np.all(np.abs(z.cpu().numpy().reshape(-1) - ref) <= LOGIT_ATOL + LOGIT_RTOL * np.abs(ref))
    assert abs(float(out3[0]) - loss_ref) < 1e-5
    got = P.from_flat(grads)
    for name, r in g_ref.items():
        assert np.abs(got[name] - r).max() <= 1e-5 * np.abs(r).max() + 1e-7, name


# bf16 math (SPWGNN_MATH_BF16) against the bf16-operand emulator: tests/test_gpu_fullsize.py.


# The chain kernels share each weight image through an LDS ring across the 4 waves of a workgroup
# (tgemm_x6_wg): no wave may exit early, a wave past the last row block runs on the clamped block and
# stores nothing. Row-block counts ≡ 1, 2, 3 (mod 4) for nodes and edges, forward + backward.
@pytest.mark.parametrize("T,N", [(5, 6), (11, 6), (27, 6), (9, 9), (3, 13)])
def test_shared_weight_ring_partial_workgroups(T, N):
    params = O.random_params(seed=23)
    obj, Rs, Rr, prop, tgt = D.synthetic_batch(T, N, seed=T + N, fully_connected=(T % 2 == 1))
    prop = np.random.default_rng(T).normal(0, 0.3, size=prop.shape).astype(np.float32)
    S = 3
    loss_ref, z_ref, g_ref = O.loss_and_grads(params, obj, Rs, Rr, prop, tgt, S)
    batch = TowerBatch.from_dense(obj, Rs, Rr, prop, device="cuda")
    print("node blocks", (batch.n_nodes + 31) // 32)
    flat, ws, z = _gpu_forward(params, batch, S, training=True, math="x6")
    out3, dz = E.bce(z, torch.tensor(tgt, device="cuda").reshape(-1), E.BceScratch("cuda"))
    grads, _ = E.backward(flat, batch, E.RunConfig(S, training=True, math="x6"), ws, dz)
    torch.cuda.synchronize()
    ref = np.asarray(z_ref).reshape(-1)
    assert np.all(np.abs(z.cpu().numpy().reshape(-1) - ref) <= LOGIT_ATOL + LOGIT_RTOL * np.abs(ref))
    assert abs(float(out3[0]) - loss_ref) < 1e-5
    got = P.from_flat(grads)
    for name, r in g_ref.items():
        assert np.abs(got[name] - r).max() <= 1e-5 * np.abs(r).max() + 1e-7, name


@pytest.mark.parametrize("math", ["x6", "f32", "bf16"])
@pytest.mark.parametrize("n_towers", [8, 3000])   # team kernels / wide kernels
def test_backward_writes_every_gradient(math, n_towers):
    """Nothing of the caller's `grads` buffer survives a backward (api.hip run_backward clears it, then
    the reductions write the 22 Keras tensors): a NaN-filled buffer must come out bitwise equal to a
    zero-filled one. Without the clear, 739 floats stayed NaN (measured on the GPU)."""
    params = O.random_params(seed=13)
    obj, Rs, Rr, prop, tgt = D.synthetic_batch(n_towers, 6, seed=21, fully_connected=False)
    batch = TowerBatch.from_dense(obj, Rs, Rr, prop, device="cuda")
    flat = P.to_flat(params, device="cuda")
    ws = E.Workspace("cuda")
    run = E.RunConfig(3, training=True, math=math)
    z = E.forward(flat, batch, run, ws)
    _, dz = E.bce(z, torch.tensor(tgt.reshape(-1), device="cuda"), E.BceScratch("cuda"))
    g_nan = torch.full_like(flat, float("nan"))
    g_zero = torch.zeros_like(flat)
    E.backward(flat, batch, run, ws, dz, grads=g_nan)
    E.backward(flat, batch, run, ws, dz, grads=g_zero)
    torch.cuda.synchronize()
    assert torch.isfinite(g_nan).all(), int((~torch.isfinite(g_nan)).sum())
    assert torch.equal(g_nan, g_zero)


@pytest.mark.parametrize("n_towers,S,math", [(8, 3, "x6"), (8, 1, "x6"), (40, 5, "bf16"), (300, 3, "x6"),
                                             (3000, 3, "x6"), (3000, 3, "bf16")])
def test_results_independent_of_workspace_contents(n_towers, S, math):
    """No kernel reads a workspace element that this forward/backward did not write first: the same
    step on a workspace pre-filled with NaN bytes and on one pre-filled with zeros gives bitwise equal
    logits, d/d'propagation' and gradients, all finite. (The fused small-batch kernels store only
    their towers' node rows, not the padding rows of the last 32-row block; the om.0 gradient stream
    once multiplied those rows' stale values by zero — a NaN survived as 300 om.0 gradient elements.)"""
    params = O.random_params(seed=13)
    obj, Rs, Rr, prop, tgt = D.synthetic_batch(n_towers, 6, seed=21, fully_connected=False)
    batch = TowerBatch.from_dense(obj, Rs, Rr, prop, device="cuda")

    def step(fill):
        flat = P.to_flat(params, device="cuda")
        ws = E.Workspace("cuda")
        run = E.RunConfig(S, training=True, math=math, dropout=0.1, seed=5)
        E.forward(flat, batch, run, ws)
        ws.buf.fill_(fill)
        z = E.forward(flat, batch, run, ws)
        _, dz = E.bce(z, torch.tensor(tgt.reshape(-1), device="cuda"), E.BceScratch("cuda"))
        g = torch.full_like(flat, float("nan"))
        _, dp = E.backward(flat, batch, run, ws, dz, grads=g, want_dprop=True)
        torch.cuda.synchronize()
        return z, g, dp

    za, ga, pa = step(255)   # 0xFFFFFFFF: NaN in every float of the workspace
    zb, gb, pb = step(0)
    assert torch.isfinite(ga).all(), int((~torch.isfinite(ga)).sum())
    assert torch.equal(za, zb) and torch.equal(pa, pb) and torch.equal(ga, gb)


@pytest.mark.parametrize("math", ["x6", "f32"])
@pytest.mark.parametrize("T,N,fully", [(3, 32, True), (4, 24, False), (9, 6, True)])
def test_receiver_block_plan_parity(T, N, fully, math):
    """Receiver-block plans (spwgnn_plan_fill_recv: one block per node; the x6 edge forward's column
    sums, k_edge_fwd_rb_x6): logits, loss and every gradient against the fp64 oracle at the fp32
    tolerance, training with S = 5, and the same towers through the default plan agree."""
    params = O.random_params(seed=17)
    obj, Rs, Rr, prop, tgt = D.synthetic_batch(T, N, seed=5, fully_connected=fully)
    S = 5
    loss_ref, z_ref, g_ref = O.loss_and_grads(params, obj, Rs, Rr, prop, tgt, S)
    dense = TowerBatch.from_dense(obj, Rs, Rr, prop, device="cuda")
    rb = TowerBatch.from_edges(obj.reshape(-1, 3), dense.tower_nodes, dense.src, dense.dst, dense.tower_edges,
                               prop.reshape(-1, 100), device="cuda", recv_blocks=True)
    assert rb.flags == 1 and rb.n_eblocks == rb.n_nodes
    zs = []
    for batch in (rb, dense):
        flat, ws, z = _gpu_forward(params, batch, S, training=True, math=math)
        out3, dz = E.bce(z, torch.tensor(tgt, device="cuda").reshape(-1), E.BceScratch("cuda"))
        grads, _ = E.backward(flat, batch, E.RunConfig(S, training=True, math=math), ws, dz)
        torch.cuda.synchronize()
        zc = z.cpu().numpy().reshape(z_ref.shape)
        assert np.all(np.abs(zc - z_ref) <= 1e-5 + 1e-5 * np.abs(z_ref)), np.abs(zc - z_ref).max()
        assert abs(float(out3[0]) - loss_ref) < 1e-5
        got = P.from_flat(grads)
        for name, ref in g_ref.items():
            assert np.abs(got[name] - ref).max() <= 1e-5 * np.abs(ref).max() + 1e-7, name
        zs.append(zc)
        # inference forward of the same plan
        zi = _gpu_forward(params, batch, S, training=False, math=math)[2].cpu().numpy().reshape(z_ref.shape)
        assert np.all(np.abs(zi - z_ref) <= 1e-5 + 1e-5 * np.abs(z_ref))
    assert np.abs(zs[0] - zs[1]).max() <= 2e-6
