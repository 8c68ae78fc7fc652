"""Does any result depend on the workspace's prior contents? Run fwd+bwd on a workspace pre-filled
with NaN bytes and on one pre-filled with zeros; report non-finite and differing gradient elements."""
import os, sys
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import model as O
from spwgnn_amd import TowerBatch, data as D, engine as E, params as P
params = O.random_params(seed=13)


def run_once(batch, tgt, fill, S, math):
    flat = P.to_flat(params, device="cuda")
    ws = E.Workspace("cuda")
    run = E.RunConfig(S, training=True, math=math, dropout=0.1, seed=5)
    E.forward(flat, batch, run, ws)
    ws.buf.fill_(fill)
    z = E.forward(flat, batch, run, ws)
    _, dz = E.bce(z, torch.tensor(tgt.reshape(-1), device="cuda"), E.BceScratch("cuda"))
    g = torch.full_like(flat, float("nan"))
    _, dp = E.backward(flat, batch, run, ws, dz, grads=g, want_dprop=True)
    torch.cuda.synchronize()
    return z.cpu().numpy(), g.cpu().numpy(), dp.cpu().numpy()


for n_towers, S, math in ((8, 3, "x6"), (8, 1, "x6"), (40, 5, "bf16"), (300, 3, "x6"), (3000, 3, "x6")):
    obj, Rs, Rr, prop, tgt = D.synthetic_batch(n_towers, 6, seed=21, fully_connected=False)
    batch = TowerBatch.from_dense(obj, Rs, Rr, prop, device="cuda")
    za, ga, pa = run_once(batch, tgt, 255, S, math)
    zb, gb, pb = run_once(batch, tgt, 0, S, math)
    bad = np.nonzero(~np.isfinite(ga) | (ga != gb))[0]
    print(f"towers {n_towers} S {S} {math}: z equal {np.array_equal(za, zb)} dprop equal {np.array_equal(pa, pb)} "
          f"grad elements non-finite or differing: {len(bad)}")
    for name, off, shape in P.layout():
        n = int(np.prod(shape))
        sel = bad[(bad >= off) & (bad < off + n)] - off
        if len(sel):
            print("   ", name, shape, len(sel), [tuple(int(x) for x in np.unravel_index(int(i), shape)) for i in sel[:6]])
