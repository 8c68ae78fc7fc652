"""Debug helper: per-tensor gradient error of the HIP backward against the oracle (small case)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from oracle import model as O
from spwgnn_amd import TowerBatch, data as D, engine as E, params as P

params = O.random_params(seed=7)
obj, Rs, Rr, prop, tgt = D.synthetic_batch(6, 6, seed=2, fully_connected=False)
S = int(sys.argv[1]) if len(sys.argv) > 1 else 5
loss_ref, z_ref, g_ref = O.loss_and_grads(params, obj, Rs, Rr, prop, tgt, S)
batch = TowerBatch.from_dense(obj, Rs, Rr, prop, device="cuda")
flat = P.to_flat(params, device="cuda")
ws = E.Workspace("cuda")
run = E.RunConfig(S, training=True)
z = E.forward(flat, batch, run, ws)
out3, dz = E.bce(z, torch.tensor(tgt, device="cuda").reshape(-1), E.BceScratch("cuda"))
grads, _ = E.backward(flat, batch, run, ws, dz)
torch.cuda.synchronize()
print("dlogit", float(np.abs(z.cpu().numpy().reshape(z_ref.shape) - z_ref).max()))
g = P.from_flat(grads)
for k, ref in g_ref.items():
    print(f"{k:14s} rel={np.abs(g[k]-ref).max()/(np.abs(ref).max()+1e-30):.3e}")
k = "rmp.0.kernel"
d = np.abs(g[k] - g_ref[k]).max(axis=1)
for lo, hi in ((0, 150), (150, 250), (250, 350)):
    print(k, lo, hi, f"{d[lo:hi].max():.3e}", f"ref {np.abs(g_ref[k][lo:hi]).max():.3e}")
