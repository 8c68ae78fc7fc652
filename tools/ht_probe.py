"""x6 gradient error against the fp64 oracle, per tensor (max |Δ| / tensor max), for small batches
run on whatever kernels the library in SPWGNN_LIB takes (build it with -DSPWGNN_TEAM_MAX_BLOCKS=0 to
put small batches on the chain kernels). usage: python3 tools/ht_probe.py"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import model as O
from spwgnn_amd import TowerBatch, data as D, engine as E, params as P

CASES = ((16, 6, True, 5, 1), (16, 6, False, 3, 2), (8, 12, True, 5, 3), (8, 12, True, 5, 3), (8, 12, True, 1, 3),
         (8, 12, False, 5, 4), (24, 12, True, 5, 5), (6, 16, True, 5, 6), (4, 7, True, 2, 7))
first = int(os.environ.get('PROBE_FIRST', 0))
for (B, N, fully, S, seed) in CASES[first:int(os.environ.get('PROBE_LAST', len(CASES)))]:
    params = O.random_params(40 + seed)
    obj, Rs, Rr, prop, tgt = D.synthetic_batch(B, N, seed=20 + seed, fully_connected=fully)
    batch = TowerBatch.from_dense(obj, Rs, Rr, prop, device="cuda")
    flat = P.to_flat(params, device="cuda")
    ws = E.Workspace("cuda")
    run = E.RunConfig(S, training=True, math="x6", dropout=0.0)
    z = E.forward(flat, batch, run, ws)
    _, dz = E.bce(z, torch.as_tensor(tgt, device="cuda").reshape(-1), E.BceScratch("cuda"))
    g, _ = E.backward(flat, batch, run, ws, dz)
    torch.cuda.synchronize()
    g = P.from_flat(g)
    loss_ref, z_ref, g_ref = O.loss_and_grads(params, obj, Rs, Rr, prop, tgt, S)
    zerr = float(np.abs(z.cpu().numpy().reshape(z_ref.shape) - z_ref).max())
    errs = {k: float(np.abs(g[k] - r).max() / np.abs(r).max()) for k, r in g_ref.items()}
    worst = sorted(errs.items(), key=lambda kv: -kv[1])[:4]
    print(f"B{B} N{N} {'fc' if fully else 'thr'} S{S}: logits {zerr:.2e}; worst grads " +
          " ".join(f"{k} {v:.2e}" for k, v in worst), flush=True)
