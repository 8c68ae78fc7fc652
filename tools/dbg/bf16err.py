"""bf16 math vs the fp64 oracle: logit and per-tensor gradient errors (sets the test tolerances)."""
import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
import numpy as np, torch
from oracle import model as O
from spwgnn_amd import TowerBatch, data as D, engine as E, params as P

for N, fully in ((6, True), (12, True), (9, False)):
    params = O.random_params(5)
    obj, Rs, Rr, prop, tgt = D.synthetic_batch(64, N, seed=2, fully_connected=fully)
    batch = TowerBatch.from_dense(obj, Rs, Rr, prop, device="cuda")
    flat = P.to_flat(params, device="cuda")
    for math in ("x6", "bf16"):
        ws = E.Workspace("cuda")
        run = E.RunConfig(5, training=True, math=math)
        z = E.forward(flat, batch, run, ws)
        out3, dz = E.bce(z, torch.tensor(tgt.reshape(-1), device="cuda"), E.BceScratch("cuda"))
        g, _ = E.backward(flat, batch, run, ws, dz)
        torch.cuda.synchronize()
        loss_ref, z_ref, g_ref = O.loss_and_grads(params, obj, Rs, Rr, prop, tgt, 5)
        zz = z.cpu().numpy().reshape(z_ref.shape)
        gg = P.from_flat(g)
        rel = {k: float(np.abs(gg[k] - g_ref[k]).max() / (np.abs(g_ref[k]).max() + 1e-30)) for k in g_ref}
        cos = min(float((gg[k] * g_ref[k]).sum() / (np.linalg.norm(gg[k]) * np.linalg.norm(g_ref[k]) + 1e-30)) for k in g_ref)
        print(f"N={N} fully={fully} {math:5s} max|dz|={np.abs(zz - z_ref).max():.3e} "
              f"max rel|dz|={(np.abs(zz - z_ref) / (np.abs(z_ref) + 1e-3)).max():.3e} "
              f"loss {float(out3[0]):.6f} vs {loss_ref:.6f}  grad max-rel {max(rel.values()):.3e} min-cos {cos:.6f}")
