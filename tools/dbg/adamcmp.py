"""Debug: trainer steps vs the oracle's Keras Adam, per math mode, per step, worst tensor."""
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
names = list(P.from_flat(P.to_flat(params, dtype=torch.float64)).keys())
for math in ["f32", "x6"]:
    flat = P.to_flat(params, device="cuda")
    tr = Trainer(flat, mp_steps=5, dropout=0.0, math=math)
    opt = O.KerasAdam()
    ref = P.to_flat(params, dtype=torch.float64).numpy()
    for step in range(3):
        tr.step(batch, torch.tensor(tgt.reshape(-1), device="cuda"))
        _, _, g = O.loss_and_grads(P.from_flat(torch.tensor(ref)), obj, Rs, Rr, prop, tgt, 5)
        gflat = P.to_flat(g, dtype=torch.float64).numpy()
        ref = opt.step(ref, gflat)
        torch.cuda.synchronize()
        got = flat.cpu().numpy()
        d = np.abs(got - ref)
        k = int(np.argmax(d))
        gt = P.from_flat(torch.tensor(d))
        worst = max(gt, key=lambda n: np.abs(gt[n]).max())
        print(f"{math} step {step}: max|dparam|={d.max():.3e} at flat {k} (tensor {worst}) ref grad there {gflat[k]:.3e}; "
              f"#>1e-6: {int((d > 1e-6).sum())} #>1e-5: {int((d > 1e-5).sum())} #>1e-4: {int((d > 1e-4).sum())} p99.9 {np.percentile(d, 99.9):.2e}")
