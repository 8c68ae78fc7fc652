"""Debug: per-tensor gradient differences (x6 / f32 vs the fp64 oracle), the Adam-test batch."""
import sys
import numpy as np
import torch
sys.path.insert(0, ".")
from oracle import model as O
from spwgnn_amd import TowerBatch, data as D, engine as E, params as P

params = O.random_params(12)
obj, Rs, Rr, prop, tgt = D.synthetic_batch(16, 6, seed=21, fully_connected=False)
batch = TowerBatch.from_dense(obj, Rs, Rr, None, device="cuda")
_, _, gref = O.loss_and_grads(params, obj, Rs, Rr, prop, tgt, 5)
for math in ["f32", "x6"]:
    flat = P.to_flat(params, device="cuda")
    ws = E.Workspace("cuda")
    run = E.RunConfig(5, training=True, math=math)
    z = E.forward(flat, batch, run, ws)
    out3, dz = E.bce(z, torch.tensor(tgt, device="cuda").reshape(-1), E.BceScratch("cuda"))
    grads, _ = E.backward(flat, batch, run, ws, dz)
    got = P.from_flat(grads)
    print("==", math)
    for name, ref in gref.items():
        g = got[name]
        d = np.abs(g - ref)
        k = int(np.argmax(d))
        small = np.abs(ref) < 1e-9
        sel = np.abs(ref) > 1e-7
        rel = d[sel] / np.abs(ref[sel])
        print(f"{name:14s} max|d|={d.max():.2e} p50|d|={np.median(d):.2e} p99|d|={np.percentile(d, 99):.2e} "
              f"rel>1e-3: {int((rel > 1e-3).sum())} rel>1e-2: {int((rel > 1e-2).sum())} max rel {rel.max() if rel.size else 0:.2e}")
