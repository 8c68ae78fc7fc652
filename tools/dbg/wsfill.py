"""Debug: does a pre-filled workspace change the gradients (uninitialized reads)?"""
import sys
import numpy as np
import torch
sys.path.insert(0, ".")
from oracle import model as O
from spwgnn_amd import TowerBatch, data as D, engine as E, params as P

params = O.random_params(12)
obj, Rs, Rr, prop, tgt = D.synthetic_batch(16, 6, seed=21, fully_connected=False)
batch = TowerBatch.from_dense(obj, Rs, Rr, None, device="cuda")
target = torch.tensor(tgt.reshape(-1), device="cuda")
flat = P.to_flat(params, device="cuda")
for math in ["f32", "x6"]:
    run = E.RunConfig(5, training=True, math=math)
    outs = []
    for fill in [0x00, 0xFF, 0x3F]:
        ws = E.Workspace("cuda")
        ws.get(E.workspace_bytes(batch, run)).fill_(fill)
        z = E.forward(flat, batch, run, ws)
        _, dz = E.bce(z, target, E.BceScratch("cuda"))
        g, _ = E.backward(flat, batch, run, ws, dz)
        outs.append(g.cpu().numpy().copy())
        print(math, hex(fill), "nan" if np.isnan(outs[-1]).any() else "ok", f"vs fill0 {np.abs(outs[-1] - outs[0]).max():.3e}")
