"""Where a replayed config-1 step's time goes: host plan build, the pinned batch copy, the graph
replay alone, and the full call (load + replay). usage: python tools/replay_probe.py [steps]"""
import json
import sys
import time

import numpy as np
import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
import bench  # noqa: E402
from spwgnn_amd import params as P  # noqa: E402
from spwgnn_amd.batch import HostPlan  # noqa: E402
from spwgnn_amd.replay import ReplayStep  # noqa: E402
from spwgnn_amd.trainer import Trainer  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 200
cfg = dict(bench.CONFIGS[1])
dev = torch.device("cuda", 0)
plans, tg, n_global = bench.make_workload(cfg, 0, dev, 1, plans=True)
plan, tgt = plans[0], tg[0]
tr = Trainer(P.to_flat(P.glorot_uniform(0), device=dev), mp_steps=cfg["S"], dropout=0.1, seed=7, math=cfg["math"])
rs = ReplayStep(plan, dev, tr.replay_body(plan.n_nodes, n_global))
for _ in range(20):
    rs(plan, tgt)
torch.cuda.synchronize()


def timed(fn):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(K):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / K * 1e3


src, dst = plan.src, plan.dst
out = {
    "full_call_ms": timed(lambda: rs(plan, tgt)),
    "replay_only_ms": timed(lambda: rs.graph.replay()),
    "load_only_ms": timed(lambda: rs.static.load(plan, tgt)),
    "plan_build_ms": timed(lambda: HostPlan.build(plan.arrays[0][:, :3], plan.tower_nodes, src, dst, plan.tower_edges,
                                                  edge_cap=30)),
    "eager_body_ms": timed(lambda: rs._issue()),
    "n_eblocks": plan.n_eblocks, "n_nodes": plan.n_nodes,
}
print(json.dumps({k: round(v, 4) if isinstance(v, float) else v for k, v in out.items()}))
