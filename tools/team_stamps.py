"""Phase stamps of the team relation encoder (workgroup 0, waves 0 and 4) over replayed config-1
steps; needs the -DSPWGNN_DIAG library (SPWGNN_LIB=tools/diag/libD.so).
usage: SPWGNN_LIB=... python tools/team_stamps.py"""
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
dev = torch.device("cuda", 0)
plans, tg, n_global = bench.make_workload(cfg, 0, dev, 1, plans=True)
plan, tgt = plans[0], tg[0]
tr = Trainer(P.to_flat(P.glorot_uniform(0), device=dev), mp_steps=cfg["S"], dropout=0.1, seed=7, math=cfg["math"])
rs = ReplayStep(plan, dev, tr.replay_body(plan.n_nodes, n_global))
lib = _lib.lib()
fn = lib.spwgnn_diag_team_stamps
fn.argtypes = [ctypes.c_void_p]
rows = []
for it in range(30):
    rs(plan, tgt)
    torch.cuda.synchronize()
    buf = (ctypes.c_ulonglong * 32)()
    fn(ctypes.addressof(buf))
    a = np.array(buf[:], dtype=np.int64).reshape(2, 16)
    if it >= 10:
        rows.append(a[:, :11] - a[0, 0])
r = np.median(np.array(rows), axis=0)
names = ["start", "layer0", "bar0", "g1", "bar1", "g2", "bar2", "g3", "bar3", "g4", "end"]
print(json.dumps({"wave0": dict(zip(names, r[0].tolist())), "wave4": dict(zip(names, r[1].tolist())),
                  "n_eblocks": plan.n_eblocks}))
