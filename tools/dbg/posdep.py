"""Debug: batch-position dependence of the forward logits (x6 vs f32)."""
import sys
import numpy as np
import torch
sys.path.insert(0, ".")
from oracle import model as O
from spwgnn_amd import TowerBatch, data as D, engine as E, params as P

N, S = 6, 5
params = O.random_params(6)
flat = P.to_flat(params, device="cuda")
raw = D.synthetic_towers(64, N, seed=17)
obj = (raw / 170).astype(np.float32)
for math in ["f32", "x6"]:
    def run(o):
        b = TowerBatch.fully_connected(o, device="cuda")
        return E.forward(flat, b, E.RunConfig(S, math=math), E.Workspace("cuda")).cpu().numpy().reshape(len(o), N)
    z1 = run(obj)
    z2 = run(obj)
    perm = np.roll(np.arange(64), 1)
    z3 = run(obj[perm])[np.argsort(perm)]
    z4 = run(obj[:24])
    z5 = run(obj[1:25])
    print(math, "repeat equal", np.array_equal(z1, z2), "roll1 equal", np.array_equal(z1, z3),
          "rows differing", int((z1 != z3).any(1).sum()), "max", float(np.abs(z1 - z3).max()),
          "prefix24", np.array_equal(z4, z1[:24]), "shift1", np.array_equal(z5, z1[1:25]))
