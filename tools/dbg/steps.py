"""Debug: x6 vs oracle gradients at the trainer's step-1 params for S = 1..5 propagation steps."""
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
flat = P.to_flat(params, device="cuda")
tr = Trainer(flat, mp_steps=5, dropout=0.0, math="f32")
tr.step(batch, target)
theta1 = flat.detach().clone()
p1 = P.from_flat(torch.tensor(theta1.cpu().numpy().astype(np.float64)))
for S in [1, 2, 3, 5]:
    _, _, gref = O.loss_and_grads(p1, obj, Rs, Rr, prop, tgt, S)
    gr = P.to_flat(gref, dtype=torch.float64).numpy()
    for prm, name in [(flat, "theta1"), (P.to_flat(params, device="cuda"), "theta0")]:
        if name == "theta0":
            _, _, g0 = O.loss_and_grads(params, obj, Rs, Rr, prop, tgt, S)
            ref = P.to_flat(g0, dtype=torch.float64).numpy()
        else:
            ref = gr
        for math in ["f32", "x6"]:
            run = E.RunConfig(S, training=True, math=math)
            ws = E.Workspace("cuda")
            z = E.forward(prm, batch, run, ws)
            _, dz = E.bce(z, target, E.BceScratch("cuda"))
            g, _ = E.backward(prm, batch, run, ws, dz)
            print(f"S={S} {name} {math}: max|g-ref| {np.abs(g.cpu().numpy() - ref).max():.3e}")
