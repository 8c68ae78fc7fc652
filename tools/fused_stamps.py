"""Phase stamps (s_memrealtime, 100 MHz) of the fused small-batch forward: workgroup 0's waves 0 and 4
over replayed config-1 steps. Needs a -DSPWGNN_DIAG library (SPWGNN_LIB=...).
Slots: 10 kernel start, 11/12 edge body start/end, 13/14 node body start/end, 15 after the step's
barrier; inside the node body 0 fragments requested, 1 W3 product done, 2 c_o product done,
3 after barrier 1, 4 o1 done, 5 after barrier 2, 6 P' done, 7 after barrier 3, 8 U' stored, 9 V' stored.
Edge body (the last step's, every block): 16 start, 17 operand split into LDS, 18 after the barrier, 19 GEMM done,
20 masks done, 21 receiver sums done; 22 edge indices in, 23 k-block 0's rows in, 24 its split stored.
usage: SPWGNN_LIB=... python tools/fused_stamps.py [S]"""
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from spwgnn_amd import _lib, params as P  # noqa: E402
from spwgnn_amd.replay import ReplayStep  # noqa: E402
from spwgnn_amd.trainer import Trainer  # noqa: E402

cfg = dict(bench.CONFIGS[1])
if len(sys.argv) > 1:
    cfg["S"] = int(sys.argv[1])   # e.g. 5: Keras fit's step count (the stamps are step 0's)
dev = torch.device("cuda", 0)
plans, tg, n_global = bench.make_workload(cfg, 0, dev, 1, plans=True)
plan, tgt = plans[0], tg[0]
tr = Trainer(P.to_flat(P.glorot_uniform(0), device=dev), mp_steps=cfg["S"], dropout=0.1, seed=7, math=cfg["math"])
rs = ReplayStep(plan, dev, tr.replay_body(plan.n_nodes, n_global))
fn = _lib.lib().spwgnn_diag_team_stamps
fn.argtypes = [ctypes.c_void_p]
rows = []
for it in range(40):
    rs(plan, tgt)
    torch.cuda.synchronize()
    buf = (ctypes.c_ulonglong * 64)()
    fn(ctypes.addressof(buf))
    a = np.array(buf[:], dtype=np.int64).reshape(2, 32)
    if it >= 10:
        rows.append((a - a[0, 10]) * 0.01)   # µs from the kernel start
r = np.median(np.array(rows), axis=0)
names = {10: "start", 11: "edge0", 12: "edge1", 13: "node0", 14: "node1", 15: "step_end", 0: "n.frag", 1: "n.W3",
         2: "n.co", 3: "n.bar1", 4: "n.o1", 5: "n.bar2", 6: "n.P'", 7: "n.bar3", 8: "n.U", 9: "n.V",
         16: "e.start", 22: "e.sd", 23: "e.rows", 24: "e.kb0", 17: "e.split", 18: "e.bar", 19: "e.gemm", 20: "e.masks",
         21: "e.sums"}
order = [10, 11, 12, 13, 0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 14, 15, 16, 22, 23, 24, 17, 18, 19, 20, 21]
print(json.dumps({f"wave{w}": {names[i]: round(float(r[w, i]), 2) for i in order} for w in (0, 1)}))
