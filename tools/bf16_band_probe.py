"""Diagnosis: the engine's bf16 math against the bf16-operand emulator on several
batch shapes — per-tensor gradient rel-L2 / band ratios and their median — plus the x6 math of the same
batch against the fp64 oracle (held to the fp32 tolerance), to tell arithmetic spread from a defect.
usage: python tools/bf16_band_probe.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from oracle import bf16 as OB, model as O  # noqa: E402
from spwgnn_amd import TowerBatch, data as D, engine as E, params as P  # noqa: E402


def train(flat, batch, tgt, S, math):
    ws = E.Workspace("cuda")
    run = E.RunConfig(S, training=True, math=math, dropout=0.0)
    z = E.forward(flat, batch, run, ws)
    out3, dz = E.bce(z, torch.as_tensor(tgt, device="cuda").reshape(-1), E.BceScratch("cuda"))
    g, _ = E.backward(flat, batch, run, ws, dz)
    torch.cuda.synchronize()
    return z.cpu().numpy().astype(np.float64), float(out3[0]), P.from_flat(g)


def probe(name, pos, sizes, src, dst, te, S=5, seed=12):
    params = O.random_params(44)
    flat = P.to_flat(params, device="cuda")
    n = int(sizes.sum())
    tgt = np.random.default_rng(seed).integers(0, 2, size=n).astype(np.float32)
    b = TowerBatch.from_edges(pos, sizes, src, dst, te, device="cuda")
    zb, lb, gb = train(flat, b, tgt, S, "bf16")
    ref, band = OB.noise_band(params, pos, src, dst, np.zeros((n, 100)), tgt, S)
    err = {k: OB.rel_l2(gb[k], r) for k, r in ref[2].items()}
    ratio = {k: err[k] / (band["g"][k] + 1e-12) for k in err}
    dz = zb - ref[1]
    zx, lx, gx = train(flat, b, tgt, S, "x6")
    l64, z64, g64 = O.loss_and_grads(params, pos, None, None, np.zeros((n, 100)), tgt, S, form="gather",
                                     src=src.astype(np.int64), dst=dst.astype(np.int64))
    gxe = max(np.abs(gx[k] - r).max() / np.abs(r).max() for k, r in g64.items())
    print(f"{name}: towers {len(sizes)} nodes {n} edges {len(src)} | bf16 logits rms {np.sqrt(np.mean(dz**2)):.2e} "
          f"(band {band['z_rms']:.2e}) | grad ratio median {np.median(list(ratio.values())):.2f} max "
          f"{max(ratio.values()):.2f} | bands median {np.median(list(band['g'].values())):.1e} | "
          f"x6 vs fp64: logits {np.abs(zx - z64).max():.1e} grads {gxe:.1e}", flush=True)
    # bf16 engine vs the fp64 oracle (no rounding) and the emulator vs the fp64 oracle
    e_eng = np.median([OB.rel_l2(gb[k], r) for k, r in g64.items()])
    e_emu = np.median([OB.rel_l2(ref[2][k], r) for k, r in g64.items()])
    print(f"    median rel-L2 to exact: engine {e_eng:.2e}, emulator {e_emu:.2e}", flush=True)


def sub(pos, sizes, src, dst, te, pick):
    off = np.concatenate([[0], np.cumsum(sizes)])
    eoff = np.concatenate([[0], np.cumsum(te)])
    P_, S_, D_, base = [], [], [], 0
    for t in pick:
        P_.append(pos[off[t]:off[t + 1]])
        S_.append(src[eoff[t]:eoff[t + 1]] - off[t] + base)
        D_.append(dst[eoff[t]:eoff[t + 1]] - off[t] + base)
        base += int(sizes[t])
    return np.concatenate(P_), sizes[pick], np.concatenate(S_), np.concatenate(D_), te[pick]


pos, sizes, src, dst, te, _ = D.ragged_batch(4096, 4, 16, seed=9)
pick = np.sort(np.random.default_rng(11).choice(4096, 24, replace=False))
probe("ragged 4-16 thr (test sub-batch shape)", *sub(pos, sizes, src, dst, te, pick))
probe("ragged 4-16 thr, 64 towers", *sub(pos, sizes, src, dst, te, np.arange(64)))
for N in (16, 12, 6):
    p2, s2, a2, b2, t2, _ = D.ragged_batch(64, N, N, seed=3)
    probe(f"uniform N={N} thr, 64 towers", p2, s2, a2, b2, t2)
p3, s3, a3, b3, t3, _ = D.ragged_batch(24, 4, 16, seed=5, threshold=None)
probe("ragged 4-16 fully connected, 24 towers", p3, s3, a3, b3, t3)
