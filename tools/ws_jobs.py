"""Per-job breakdown of the batched weight gradient: every k_wgrad_ws job run as
its own launch (SPWGNN_WS_UNBATCHED=1), timed with HIP events around each launch, with its own
roofs — algorithmic FLOPs against the math's matrix peak, padded MFMA cycles at the measured clock,
and compulsory operand bytes (each X and Y row read once) against 8 TB/s.
usage: python tools/ws_jobs.py [config] [steps]   (config 0 = the headline, 3 = bf16 N=12)"""
import json
import os
import sys

os.environ["SPWGNN_WS_UNBATCHED"] = "1"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from spwgnn_amd import _lib, params as P  # noqa: E402
from spwgnn_amd.trainer import Trainer  # noqa: E402

cfg_id = int(sys.argv[1]) if len(sys.argv) > 1 else 0
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
cfg = dict(bench.CONFIGS[cfg_id])
dev = torch.device("cuda", 0)
batches, targets, n_global = bench.make_workload(cfg, 0, dev, 1)
S, math = cfg["S"], cfg["math"]
tr = Trainer(P.to_flat(P.glorot_uniform(0), device=dev), mp_steps=S, dropout=0.1, seed=7, math=math)
step_in = ((batches[0], targets[0]) if len(batches) == 1 else (batches, targets)) + (n_global,)
for _ in range(2):
    tr.step(*step_in)
torch.cuda.synchronize()
ms, per_step, _ = bench.timed_steps(tr, step_in, _lib.K_WGRAD_WS, len(batches), steps, bench.MAX_LAUNCHES)
ms = np.array(ms).reshape(steps * len(batches), -1).mean(0)
Ne = sum(b.n_edges for b in batches) / len(batches)
Nn = sum(b.n_nodes for b in batches) / len(batches)
b16 = math == "bf16"
e = 2 if b16 else 4          # bytes per stored element of a bf16-stored edge operand (§3g)
# (name, rows, FLOPs per row, X bytes per row, Y bytes per row, padded KX, padded NY)
jobs = [
    ("rm.1 [z1|1]ᵀdz2", Ne, 2 * 151 * 150, 8, 152 * e, 160, 160),
    ("rm.2 [z2|1]ᵀdz3", Ne, 2 * 151 * 150, 152 * e, 152 * e, 160, 160),
    ("rm.3 [z3|1]ᵀdz4", Ne, 2 * 151 * 150, 152 * e, 152 * e, 160, 160),
    ("W1a [cr|1]ᵀdA", Ne, 2 * 151 * 150, 152 * e, 160 * e, 160, 160),
    ("W1b Pᵀ dU", Nn * S, 2 * 100 * 150, 416, 608, 128, 160),
    ("W1c Pᵀ dV", Nn * S, 2 * 100 * 150, 416, 608, 128, 160),
    ("omp0.P Pᵀ do1", Nn * S, 2 * 100 * 100, 416, 416, 128, 128),
    ("omp0.a aᵀ do1", Nn * S, 2 * 100 * 100, 416, 416, 128, 128),
    ("W3 [H2s|deg]ᵀ g", Nn * S, 2 * 151 * 100, 608, 416, 160, 128),
    ("omp0.c [co|1]ᵀ Σdo1", Nn, 2 * 101 * 100, 416, 416, 128, 128),
    ("omp1 [o1|1]ᵀ dx", Nn * S, 2 * 101 * 101, 416, 416, 128, 128),
    ("om.1 [zo1|1]ᵀ dzo2", Nn, 2 * 101 * 100, 16, 416, 128, 128),
]
peak = bench.MATH_PEAK[math]
parts = 1 if b16 else 6
clock = float(os.environ.get("CLOCK_GHZ", "2.06"))
out = []
tot_ms = 0.0
print(f"config {cfg_id} ({math}): Ne={Ne:.0f} Nn={Nn:.0f} S={S}; {len(ms)} launches per micro-batch")
print(f"{'job':22s} {'ms':>7s} {'TF/s':>7s} {'frac':>6s} {'mfma_ms':>8s} {'GB':>6s} {'GB/s':>7s} {'hbm_ms':>7s}")
for (name, rows, fl, xb, yb, kx, ny), t in zip(jobs, ms):
    flops = rows * fl
    nbytes = rows * (xb + yb)
    # padded MFMA cycles: (kx/16)(ny/16) 16x16x32 tiles × parts products × 16 cycles per 32 rows, 4 SIMDs per CU
    mf_ms = rows / 32 * (kx // 16) * (ny // 16) * parts * 16 / 4 / 256 / (clock * 1e9) * 1e3
    r = dict(job=name, ms=round(float(t), 4), tflops=round(flops / t / 1e9, 1), frac=round(flops / t / 1e9 / peak, 3),
             mfma_floor_ms=round(mf_ms, 4), gbytes=round(nbytes / 1e9, 3), gbs=round(nbytes / t / 1e6, 0),
             hbm_floor_ms=round(nbytes / 8e12 * 1e3, 4))
    out.append(r)
    tot_ms += t
    print(f"{name:22s} {t:7.3f} {r['tflops']:7.1f} {r['frac']:6.3f} {mf_ms:8.3f} {r['gbytes']:6.2f} {r['gbs']:7.0f} "
          f"{r['hbm_floor_ms']:7.3f}")
print(f"sum {tot_ms:.3f} ms")
print(json.dumps({"config": cfg_id, "math": math, "clock_ghz_assumed": clock, "jobs": out, "sum_ms": round(tot_ms, 4)}))
