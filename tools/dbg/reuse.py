"""Debug: gradients at the same params from a fresh vs a reused workspace (x6 / f32)."""
import sys
import numpy as np
import torch
sys.path.insert(0, ".")
from oracle import model as O
from spwgnn_amd import TowerBatch, data as D, engine as E, params as P

params = O.random_params(12)
params2 = O.random_params(13)
obj, Rs, Rr, prop, tgt = D.synthetic_batch(16, 6, seed=21, fully_connected=False)
batch = TowerBatch.from_dense(obj, Rs, Rr, None, device="cuda")
_, _, gref = O.loss_and_grads(params2, obj, Rs, Rr, prop, tgt, 5)
def grads(math, ws, prm):
    flat = P.to_flat(prm, device="cuda")
    run = E.RunConfig(5, training=True, math=math)
    z = E.forward(flat, batch, run, ws)
    out3, dz = E.bce(z, torch.tensor(tgt, device="cuda").reshape(-1), E.BceScratch("cuda"))
    g, _ = E.backward(flat, batch, run, ws, dz)
    return P.from_flat(g)
for math in ["f32", "x6"]:
    fresh = grads(math, E.Workspace("cuda"), params2)
    ws = E.Workspace("cuda")
    grads(math, ws, params)
    reused = grads(math, ws, params2)
    for name in gref:
        a, b, r = fresh[name], reused[name], gref[name]
        print(f"{math} {name:14s} fresh-vs-reused {np.abs(a - b).max():.3e}  fresh-vs-ref {np.abs(a - r).max():.3e} reused-vs-ref {np.abs(b - r).max():.3e}")
