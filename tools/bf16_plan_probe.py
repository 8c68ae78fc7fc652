"""Diagnosis: bf16 math on one batch through the default and the receiver-block plan, each against the
bf16-operand emulator band (tests/test_gpu_fullsize.py's check, printed instead of asserted).
usage: python tools/bf16_plan_probe.py [T N fully]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from oracle import bf16 as OB, model as O  # noqa: E402
from spwgnn_amd import TowerBatch, data as D, engine as E, params as P  # noqa: E402

T, N, fully = (int(sys.argv[1]), int(sys.argv[2]), sys.argv[3] == "1") if len(sys.argv) > 3 else (6, 24, False)
params = O.random_params(17)
obj, Rs, Rr, prop, tgt = D.synthetic_batch(T, N, seed=5, fully_connected=fully)
dense = TowerBatch.from_dense(obj, Rs, Rr, prop, device="cuda")
rb = TowerBatch.from_edges(obj.reshape(-1, 3), dense.tower_nodes, dense.src, dense.dst, dense.tower_edges,
                           prop.reshape(-1, 100), device="cuda", recv_blocks=True)
e = np.array(O.dense_to_edges(Rs, Rr), np.int64).reshape(-1, 4)
src, dst = e[:, 0] * N + e[:, 2], e[:, 0] * N + e[:, 3]
ref, band = OB.noise_band(params, obj.reshape(-1, 3), src, dst, prop.reshape(-1, 100), tgt.reshape(-1), 5)
flat = P.to_flat(params, device="cuda")
for name, b in (("default", dense), ("recv", rb)):
    for training in (True,):
        ws = E.Workspace("cuda")
        run = E.RunConfig(5, training=True, math="bf16")
        z = E.forward(flat, b, run, ws)
        out3, dz = E.bce(z, torch.as_tensor(tgt, device="cuda").reshape(-1), E.BceScratch("cuda"))
        g, _ = E.backward(flat, b, run, ws, dz)
        torch.cuda.synchronize()
        g = P.from_flat(g)
        dzz = z.cpu().numpy().astype(np.float64) - ref[1]
        ratio = {k: OB.rel_l2(g[k], r) / (band["g"][k] + 1e-12) for k, r in ref[2].items()}
        print(f"{name} nw_max {b.nw_max} flags {b.flags}: logits rms {np.sqrt(np.mean(dzz**2)):.2e} (band {band['z_rms']:.2e}) "
              f"grad ratio median {np.median(list(ratio.values())):.2f} max {max(ratio.values()):.2f} "
              + " ".join(f"{k}={v:.2f}" for k, v in ratio.items()), flush=True)
