"""Dump logits + every gradient of one training fwd/bwd per batch shape and math (library from
SPWGNN_LIB) so two builds can be compared bitwise (tools/cmp_npz.py): small batches (≤ 512 wave-tiles:
the fused small-batch kernels), wide ones (n6w, n12w) and a ragged bf16 one.
usage python tools/b16_dump.py OUT.npz"""
import sys
import os
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import model as O
from spwgnn_amd import TowerBatch, data as D, engine as E, params as P

out = {}
params = O.random_params(7)
flat = P.to_flat(params, device="cuda")
shapes = {"n12": (512, 12, True), "n6": (1024, 6, False), "n6w": (4096, 6, True), "n12w": (2048, 12, True)}
for name, (B, N, fully) in shapes.items():
    obj, Rs, Rr, prop, tgt = D.synthetic_batch(B, N, seed=3, fully_connected=fully)
    batch = TowerBatch.from_dense(obj, Rs, Rr, prop, device="cuda")
    for math in ("bf16", "x6"):
        run = E.RunConfig(5, training=True, math=math, dropout=0.1, seed=11)
        ws = E.Workspace("cuda")
        z = E.forward(flat, batch, run, ws)
        _, dz = E.bce(z, torch.tensor(tgt.reshape(-1), device="cuda"), E.BceScratch("cuda"))
        g, _ = E.backward(flat, batch, run, ws, dz)
        torch.cuda.synchronize()
        out[f"{name}_{math}_z"] = z.cpu().numpy()
        out[f"{name}_{math}_g"] = g.cpu().numpy()
pos, sz, s, d, te, _ = D.ragged_batch(2000, 4, 16, seed=5)
rag = TowerBatch.from_edges(pos, sz, s, d, te, device="cuda")
tg = np.random.default_rng(1).integers(0, 2, size=int(sz.sum())).astype(np.float32)
run = E.RunConfig(5, training=True, math="bf16", dropout=0.1, seed=12)
ws = E.Workspace("cuda")
z = E.forward(flat, rag, run, ws)
_, dz = E.bce(z, torch.tensor(tg, device="cuda"), E.BceScratch("cuda"))
g, _ = E.backward(flat, rag, run, ws, dz)
torch.cuda.synchronize()
out["rag_bf16_z"] = z.cpu().numpy()
out["rag_bf16_g"] = g.cpu().numpy()
np.savez(sys.argv[1], **out)
print("dumped", sys.argv[1], len(out))
