"""Run-to-run determinism of one training forward + backward on a bench config's workload: the same
batch, parameters and dropout key twice in one process; prints the logits and every gradient tensor
that are not bitwise equal. usage: [SPWGNN_LIB=...] python tools/determinism.py [CONFIG] [REPEATS]"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from spwgnn_amd import engine as E, params as P  # noqa: E402

c = int(sys.argv[1]) if len(sys.argv) > 1 else 2
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
cfg = dict(bench.CONFIGS[c])
dev = torch.device("cuda", 0)
batches, targets, n_global = bench.make_workload(cfg, 0, dev, 1)
batch, tgt = batches[0], targets[0]
flat = P.to_flat(P.glorot_uniform(0), device=dev)
run = E.RunConfig(cfg["S"], training=True, math=cfg["math"], dropout=0.1, seed=5)
outs = []
for r in range(reps):
    ws = E.Workspace(dev)
    z = E.forward(flat, batch, run, ws)
    _, dz = E.bce(z, tgt, E.BceScratch(dev))
    g = E.backward(flat, batch, run, ws, dz)
    g = g[0] if isinstance(g, tuple) else g
    torch.cuda.synchronize()
    outs.append((z.clone(), g.clone()))
z0, g0 = outs[0]
for r in range(1, reps):
    z, g = outs[r]
    dz_ = (z != z0).sum().item()
    print(f"rep {r}: logits differing {dz_} of {z.numel()}, max|d| {float((z - z0).abs().max()):.3e}")
    for name, o, shape in P.layout():
        n = int(np.prod(shape))
        a, b = g0[o:o + n], g[o:o + n]
        if not torch.equal(a, b):
            print(f"   {name}: {(a != b).sum().item()} of {n} differ, max|d| {float((a - b).abs().max()):.3e}")
    print(f"   grads differing {(g != g0).sum().item()} of {g.numel()}")
