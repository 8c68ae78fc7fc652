"""Replayable training steps: forward → BCE → backward → Adam captured once into a hipGraph and
replayed for every later batch of the same geometry.

The reference trains with Keras fit at batch 32 (src/main.py:92-98). At that size a step is ~50
small kernel launches; a replayed step issues the whole sequence as one graph launch, so the host
only prepares the next batch (measured on MI355X, BASELINE config 1: the replayed step is the
kernels' own 0.40 ms — the small-batch kernels' latency, not launch overhead, is what remains;
DESIGN.md §3k). What a capture bakes in, and how it stays valid:

* sizes — the batch is planned with per-tower block capacity N(N−1) (spwgnn_plan_fill_cap), so
  every batch of B towers of N boxes has the same wave-tiles and blocks whatever its relations
  (unused capacity is padding, index −1, which matches no node);
* addresses — the batch arrays and targets live in static device buffers that each step refills
  with ONE pinned host→device copy before the replay; workspace, BCE scratch, logits, dlogits and
  gradients belong to the step object;
* per-step scalars — the dropout key and the Adam step count are device words advanced by
  spwgnn_step_advance at the start of each step; lr_t comes from a host-built table
  (spwgnn_adam_lr_table, the expression spwgnn_adam evaluates).

The first call of a geometry runs the step eagerly (a real step), then captures it; `graph=False`
runs the identical launch sequence eagerly every time, so replayed and eager training agree bit
for bit (tests/test_gpu_replay.py).
"""
from __future__ import annotations

from typing import Callable, Dict, Optional

import numpy as np
import torch

from . import _lib, engine as E
from .batch import HostPlan, TowerBatch

# Adam steps covered by one lr table (4 MiB); later steps read the last entry, which is exact: lr_t
# = lr·sqrt(1−β2^t)/(1−β1^t) equals lr in fp32 from t ≈ 2·10^4 on (β2 = 0.999)
LR_TABLE_LEN = 1 << 20


def _i64(x: int) -> int:
    x &= 0xFFFFFFFFFFFFFFFF
    return x - (1 << 64) if x >= (1 << 63) else x


class DeviceCounters:
    """The device words a replayable step reads: the dropout key (int64) and the Adam step count
    (int32), with the lr table of the optimizer's (lr, β1, β2)."""

    def __init__(self, device, key: int, step: int, lr: float, beta1: float, beta2: float):
        self.device = torch.device(device)
        self.key = torch.tensor([_i64(key)], dtype=torch.int64, device=self.device)
        self.step = torch.tensor([int(step)], dtype=torch.int32, device=self.device)
        self.lr_table = E.adam_lr_table(LR_TABLE_LEN, lr, beta1, beta2, self.device)
        self.hyper = (float(lr), float(beta1), float(beta2))

    def set(self, key: Optional[int] = None, step: Optional[int] = None, lr: Optional[float] = None,
            beta1: Optional[float] = None, beta2: Optional[float] = None):
        """Host values → device words (stream-ordered copies; outside any capture). A changed
        (lr, β1, β2) rebuilds the lr table IN PLACE: captured graphs keep reading its address."""
        if key is not None:
            self.key.fill_(_i64(key))
        if step is not None:
            self.step.fill_(int(step))
        hyper = (float(self.hyper[0] if lr is None else lr), float(self.hyper[1] if beta1 is None else beta1),
                 float(self.hyper[2] if beta2 is None else beta2))
        if hyper != self.hyper:
            self.lr_table.copy_(E.adam_lr_table(LR_TABLE_LEN, *hyper, self.device))
            self.hyper = hyper


class StaticBatch:
    """A batch geometry's device arrays at fixed addresses, refilled per step in one copy."""

    def __init__(self, plan: HostPlan, device):
        self.device = torch.device(device)
        self.geometry = plan.geometry
        self.offsets, total = [], 0
        for a in plan.arrays:
            self.offsets.append(total)
            total += (a.nbytes + 15) // 16 * 16
        self.n_target = plan.n_nodes
        self.t_off = total
        total += plan.n_nodes * 4
        self.total = max(total, 16)
        self.buf = torch.zeros(self.total, dtype=torch.uint8, device=self.device)
        views = []
        for a, o in zip(plan.arrays, self.offsets):
            dt = torch.from_numpy(a[:0].reshape(-1)).dtype
            views.append(self.buf[o:o + a.nbytes].view(dt).view(a.shape))
        self.target = self.buf[self.t_off:self.t_off + 4 * plan.n_nodes].view(torch.float32)
        self.batch = TowerBatch.from_plan(plan, self.device, dev_arrays=views)
        # pinned staging ring: a slot is refilled only after the copy that last read it has run
        # (its event), so the host never waits on the step in flight and never allocates per step
        self.ring = [torch.empty(self.total, dtype=torch.uint8, pin_memory=True) for _ in range(self.RING)]
        self.ring_ev = [None] * self.RING
        self.loads = 0

    RING = 3

    def load(self, plan: HostPlan, target: np.ndarray):
        """This step's plan arrays and targets → the static buffers (one pinned staging slot, one
        non-blocking copy on the current stream)."""
        if plan.geometry != self.geometry:
            raise ValueError("batch geometry differs from the captured one")
        slot = self.loads % self.RING
        self.loads += 1
        if self.ring_ev[slot] is not None:
            self.ring_ev[slot].synchronize()
        host = self.ring[slot]
        hv = host.numpy()
        for a, o in zip(plan.arrays, self.offsets):
            hv[o:o + a.nbytes] = np.ascontiguousarray(a).reshape(-1).view(np.uint8)
        t = np.ascontiguousarray(target, np.float32).reshape(-1)
        if t.size != self.n_target:
            raise ValueError("one target per node")
        hv[self.t_off:self.t_off + t.nbytes] = t.view(np.uint8)
        self.buf.copy_(host, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(self.device))
        self.ring_ev[slot] = ev
        # host-side copies the wrappers keep for reporting (edge ids, counts) follow the new batch
        b = self.batch
        b.tower_edges, b.src, b.dst, b.edge_id = plan.tower_edges, plan.src, plan.dst, plan.edge_id
        b.tower_nodes, b.node_shape = plan.tower_nodes, plan.node_shape


class ReplayStep:
    """One batch geometry's training step (forward, BCE, backward, Adam) as a replayed hipGraph.

    `body(batch, target, ws, bce, z, dz)` issues the step's launches on the current stream; it is
    run eagerly on the first call (a real step) and captured right after, then replayed."""

    def __init__(self, plan: HostPlan, device, body: Callable, graph: bool = True):
        self.static = StaticBatch(plan, device)
        self.device = self.static.device
        self.ws = E.Workspace(self.device)
        self.bce = E.BceScratch(self.device)
        n = plan.n_nodes
        self.z = torch.empty(n, dtype=torch.float32, device=self.device)
        self.dz = torch.empty(n, dtype=torch.float32, device=self.device)
        self.body = body
        self.use_graph = graph
        self.graph: Optional[torch.cuda.CUDAGraph] = None
        self.replays = 0

    def _issue(self):
        self.body(self.static.batch, self.static.target, self.ws, self.bce, self.z, self.dz)

    def __call__(self, plan: HostPlan, target: np.ndarray):
        self.static.load(plan, target)
        if self.graph is not None:
            self.graph.replay()
            self.replays += 1
            return
        self._issue()
        if self.use_graph:
            g = torch.cuda.CUDAGraph()
            # capture on torch's side stream; the eager step above already sized every buffer
            torch.cuda.current_stream(self.device).synchronize()
            with torch.cuda.graph(g):
                self._issue()
            self.graph = g


class ReplayCache:
    """ReplaySteps keyed by batch geometry (full batches and the epoch's last partial batch)."""

    def __init__(self, device, make_body: Callable[[], Callable], graph: bool = True, max_entries: int = 8):
        self.device, self.make_body, self.graph, self.max_entries = device, make_body, graph, max_entries
        self.steps: Dict[tuple, ReplayStep] = {}

    def __call__(self, plan: HostPlan, target: np.ndarray):
        key = plan.geometry
        st = self.steps.get(key)
        if st is None:
            if len(self.steps) >= self.max_entries:       # bounded: drop the oldest geometry
                self.steps.pop(next(iter(self.steps)))
            st = self.steps[key] = ReplayStep(plan, self.device, self.make_body(), self.graph)
        st(plan, target)
        return st


def step_key_mode(kind: str) -> int:
    return {"counter": _lib.STEP_KEY_COUNTER, "splitmix": _lib.STEP_KEY_SPLITMIX}[kind]
