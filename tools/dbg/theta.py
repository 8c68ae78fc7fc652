"""Debug: compare the params after one trainer step (f32 vs x6) and their gradients' padding."""
import sys
import numpy as np
import torch
sys.path.insert(0, ".")
from oracle import model as O
from spwgnn_amd import TowerBatch, data as D, engine as E, params as P
from spwgnn_amd import _lib

params = O.random_params(12)
obj, Rs, Rr, prop, tgt = D.synthetic_batch(16, 6, seed=21, fully_connected=False)
batch = TowerBatch.from_dense(obj, Rs, Rr, None, device="cuda")
target = torch.tensor(tgt.reshape(-1), device="cuda")
th = {}
from spwgnn_amd.trainer import Trainer
real = np.zeros(P.flat_size(), bool)
for name, off, shape in P.layout():
    real[off:off + int(np.prod(shape))] = True
for math in ["f32", "x6"]:
    flat = P.to_flat(params, device="cuda")
    tr = Trainer(flat, mp_steps=5, dropout=0.0, math=math)
    tr.step(batch, target)
    th[math] = flat.cpu().numpy().copy()
    g = tr.engine.grads.cpu().numpy()
    print(math, "nan params", int(np.isnan(th[math]).sum()), "max |param|", float(np.abs(th[math]).max()),
          "grad entries nonzero", int((g != 0).sum()), "of", g.size)
d = np.abs(th["x6"] - th["f32"])
k = np.argsort(d)[-5:]
print("max diff", d.max(), "at", k, th["x6"][k], th["f32"][k])
print("real mask available:", real.any())
if real.any():
    print("padding nonzero f32", int((th["f32"][~real] != 0).sum()), "x6", int((th["x6"][~real] != 0).sum()))
