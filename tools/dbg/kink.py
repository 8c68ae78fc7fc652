"""Debug: gradients at the x6 trainer's step-1 params, both maths vs the oracle (relu-kink check)."""
import sys
import numpy as np
import torch
sys.path.insert(0, ".")
from oracle import model as O
from spwgnn_amd import TowerBatch, data as D, engine as E, params as P
from spwgnn_amd.trainer import Trainer

params = O.random_params(12)
obj, Rs, Rr, prop, tgt = D.synthetic_batch(16, 6, seed=21, fully_connected=False)
batch = TowerBatch.from_dense(obj, Rs, Rr, None, device="cuda")
target = torch.tensor(tgt.reshape(-1), device="cuda")
for src in ["x6", "x6+eps", "x6-eps"]:
    flat = P.to_flat(params, device="cuda")
    Trainer(flat, mp_steps=5, dropout=0.0, math="x6").step(batch, target)
    if src != "x6":
        flat.mul_(1 + (1e-6 if src == "x6+eps" else -1e-6))
    p1 = P.from_flat(torch.tensor(flat.cpu().numpy().astype(np.float64)))
    _, _, gref = O.loss_and_grads(p1, obj, Rs, Rr, prop, tgt, 5)
    gr = P.to_flat(gref, dtype=torch.float64).numpy()
    for math in ["f32", "x6"]:
        run = E.RunConfig(5, training=True, math=math)
        ws = E.Workspace("cuda")
        z = E.forward(flat, batch, run, ws)
        _, dz = E.bce(z, target, E.BceScratch("cuda"))
        g, _ = E.backward(flat, batch, run, ws, dz)
        print(f"params from {src} step, {math} backward: max|g-ref| {np.abs(g.cpu().numpy() - gr).max():.3e}")
