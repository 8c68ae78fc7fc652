"""Debug: gradients at the trainer's step-1 params — fresh workspace vs the trainer's engine vs oracle."""
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
for math in ["f32", "x6"]:
    flat = P.to_flat(params, device="cuda")
    tr = Trainer(flat, mp_steps=5, dropout=0.0, math=math)
    tr.step(batch, target)
    theta1 = flat.detach().clone()
    # trainer engine (reused workspace / grads buffer)
    run = tr.run_config()
    z = tr.engine.forward(flat, batch, run)
    _, dz = tr.engine.loss(z, target)
    g_tr = tr.engine.backward(flat, batch, run, dz).cpu().numpy().copy()
    # fresh
    ws = E.Workspace("cuda")
    run2 = E.RunConfig(5, training=True, math=math)
    z2 = E.forward(theta1, batch, run2, ws)
    _, dz2 = E.bce(z2, target, E.BceScratch("cuda"))
    g_fr, _ = E.backward(theta1, batch, run2, ws, dz2)
    g_fr = g_fr.cpu().numpy()
    _, _, gref = O.loss_and_grads(P.from_flat(torch.tensor(theta1.cpu().numpy().astype(np.float64))), obj, Rs, Rr, prop, tgt, 5)
    gr = P.to_flat(gref, dtype=torch.float64).numpy()
    tp = O.to_torch(P.from_flat(torch.tensor(theta1.cpu().numpy().astype(np.float64))))
    zref = O.forward_dense(tp, torch.tensor(obj, dtype=torch.float64), torch.tensor(Rs, dtype=torch.float64),
                           torch.tensor(Rr, dtype=torch.float64), torch.zeros(obj.shape[0], obj.shape[1], 100, dtype=torch.float64), 5).numpy().reshape(-1)
    print(f"{math}: logits vs oracle max {np.abs(z2.cpu().numpy().reshape(-1) - zref).max():.3e}")
    gt = P.from_flat(torch.tensor(g_fr))
    for name in gref:
        d = np.abs(np.asarray(gt[name]) - gref[name])
        print(f"   {name:14s} max|g| {np.abs(gref[name]).max():.2e} max|d| {d.max():.2e}")
    print(f"{math}: z trainer vs fresh max {float((z - z2).abs().max()):.3e}; grads trainer-vs-fresh {np.abs(g_tr - g_fr).max():.3e}, "
          f"fresh-vs-oracle {np.abs(g_fr - gr).max():.3e}, trainer-vs-oracle {np.abs(g_tr - gr).max():.3e}")
