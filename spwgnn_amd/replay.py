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
  from a pinned staging slot inside its forward's first launch (spwgnn_run.prologue, for a body
  that takes `pre`; otherwise a spwgnn_copy_in kernel of its own); workspace, BCE scratch, logits,
  dlogits and gradients belong to the step object;
* per-step scalars — the dropout key and the Adam step count are device words advanced at the
  start of each step (the same prologue, or spwgnn_step_advance); lr_t comes from a host-built
  table (spwgnn_adam_lr_table, the expression spwgnn_adam evaluates).

The first call of a geometry runs the step eagerly (a real step), then captures it; `graph=False`
runs the identical launch sequence eagerly every time, so replayed and eager training agree bit
for bit (tests/test_gpu_replay.py).
"""
from __future__ import annotations

import ctypes as C
import inspect
import os
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


def _mapped_device_ptr(host: torch.Tensor) -> int:
    """The device address of a pinned host tensor (spwgnn_host_device_ptr): kernels read it over
    PCIe. Raises if the allocation is not device-mapped (the kernel would fault)."""
    return _lib.host_device_ptr(host.data_ptr())


class StaticBatch:
    """A batch geometry's device arrays at fixed addresses, refilled per step from pinned staging.

    Two pinned (device-mapped) staging slots: the host writes the next step's arrays into one while
    the step that reads the other runs; `copy_in(slot)` moves a slot into the device buffer with one
    kernel (spwgnn_copy_in) on the current stream — inside a captured step it is the graph's first
    kernel node, so no copy sits between two replays."""

    SLOTS = 2

    def __init__(self, plan: HostPlan, device):
        self.device = torch.device(device)
        self.geometry = plan.geometry
        self.offsets, total = [], 0
        for a in plan.arrays:
            self.offsets.append(total)
            total += (a.nbytes + 15) // 16 * 16
        self.n_target = plan.n_nodes
        self.t_off = total
        total += (plan.n_nodes * 4 + 15) // 16 * 16
        self.total = max(total, 16)
        self.buf = torch.zeros(self.total, dtype=torch.uint8, device=self.device)
        views = []
        for a, o in zip(plan.arrays, self.offsets):
            dt = torch.from_numpy(a[:0].reshape(-1)).dtype
            views.append(self.buf[o:o + a.nbytes].view(dt).view(a.shape))
        self.target = self.buf[self.t_off:self.t_off + 4 * plan.n_nodes].view(torch.float32)
        self.batch = TowerBatch.from_plan(plan, self.device, dev_arrays=views)
        self.ring = [torch.zeros(self.total, dtype=torch.uint8, pin_memory=True) for _ in range(self.SLOTS)]
        self.ring_dev = [_mapped_device_ptr(r) for r in self.ring]
        self.loads = 0

    def fill(self, plan: HostPlan, target: np.ndarray, slot: int):
        """This step's plan arrays and targets → pinned staging slot `slot` (host writes only: the
        caller has made sure no step still reads that slot)."""
        if plan.geometry != self.geometry:
            raise ValueError("batch geometry differs from the captured one")
        hv = self.ring[slot].numpy()
        for a, o in zip(plan.arrays, self.offsets):
            hv[o:o + a.nbytes] = np.ascontiguousarray(a).reshape(-1).view(np.uint8)
        t = np.ascontiguousarray(target, np.float32).reshape(-1)
        if t.size != self.n_target:
            raise ValueError("one target per node")
        hv[self.t_off:self.t_off + t.nbytes] = t.view(np.uint8)
        self.loads += 1
        # host-side copies the wrappers keep for reporting (edge ids, counts) follow the new batch
        b = self.batch
        b.tower_edges, b.src, b.dst, b.edge_id = plan.tower_edges, plan.src, plan.dst, plan.edge_id
        b.tower_nodes, b.node_shape = plan.tower_nodes, plan.node_shape

    def copy_in(self, slot: int):
        E.copy_in(self.ring[slot], self.buf, self.total, src_dev_ptr=self.ring_dev[slot])

    def load(self, plan: HostPlan, target: np.ndarray):
        """fill + copy_in through slot 0, synchronously ordered on the current stream (tools/tests)."""
        torch.cuda.current_stream(self.device).synchronize()
        self.fill(plan, target, 0)
        self.copy_in(0)


class SlotEvent:
    """The host's "this staging slot is free again" marker: a HIP event created with
    hipEventDisableSystemFence (and no timing). The host only needs to know that the step which read
    the slot has finished — its reads of pinned memory are complete when its kernels are — so the
    system-scope release a default event performs when it is reached (an L2 write-back between two
    steps) buys nothing here. `SPWGNN_SLOT_EVENT_FENCE=1` (A/B) uses the default flags."""

    FLAGS = 0x2 | 0x20000000   # hipEventDisableTiming | hipEventDisableSystemFence

    def __init__(self):
        self.hip = _lib.hip_runtime()
        flags = 0x2 if os.environ.get("SPWGNN_SLOT_EVENT_FENCE", "0") not in ("", "0") else self.FLAGS
        h = C.c_void_p()
        st = self.hip.hipEventCreateWithFlags(C.byref(h), C.c_uint(flags))
        if st != 0:
            raise _lib.SpwgnnError(f"hipEventCreateWithFlags failed ({st})")
        self.h = h

    def record(self, stream: torch.cuda.Stream) -> None:
        st = self.hip.hipEventRecord(self.h, C.c_void_p(stream.cuda_stream))
        if st != 0:
            raise _lib.SpwgnnError(f"hipEventRecord failed ({st})")

    def synchronize(self) -> None:
        st = self.hip.hipEventSynchronize(self.h)
        if st != 0:
            raise _lib.SpwgnnError(f"hipEventSynchronize failed ({st})")

    def __del__(self):
        try:
            self.hip.hipEventDestroy(self.h)
        except Exception:
            pass


class ReplayStep:
    """One batch geometry's training step (forward, BCE, backward, Adam) as a replayed hipGraph.

    `body(batch, target, ws, bce, z, dz)` issues the step's launches on the current stream; it is
    run eagerly on the first call (a real step) and captured right after, then replayed.

    The batch upload is part of the step: its first kernel copies a pinned staging slot into the
    static device buffer (StaticBatch.copy_in). Two slots, one graph each: step i reads slot i mod 2,
    and the host fills slot i mod 2 once step i − 2, its last reader, has finished — so the host
    prepares a batch while the previous step runs, and the GPU never waits on a DMA copy between two
    replays (that copy left it idle ≈ 26 µs per Keras-fit step at batch 32,
    profiles/r04_fit_step_gaps.txt)."""

    def __init__(self, plan: HostPlan, device, body: Callable, graph: bool = True):
        self.static = StaticBatch(plan, device)
        self.device = self.static.device
        self.ws = E.Workspace(self.device)
        self.bce = E.BceScratch(self.device)
        n = plan.n_nodes
        self.z = torch.empty(n, dtype=torch.float32, device=self.device)
        self.dz = torch.empty(n, dtype=torch.float32, device=self.device)
        self.body = body
        # a body taking `pre` gets the upload as a prologue of its forward's first launch
        self.fold = E.FOLD_PROLOGUE and "pre" in inspect.signature(body).parameters
        self.use_graph = graph
        self.graphs: list = [None] * StaticBatch.SLOTS
        self.done: list = [None] * StaticBatch.SLOTS   # per slot: SlotEvent after the last step that read it
        self.calls = 0
        self.replays = 0

    @property
    def graph(self) -> Optional[torch.cuda.CUDAGraph]:
        return self.graphs[0]

    def _issue(self, k: int):
        st = self.static
        if self.fold:   # the body's forward runs the upload in its first launch (spwgnn_run.prologue)
            pre = E.Prologue(dst=st.buf, src_dev_ptr=st.ring_dev[k], nbytes=st.total)
            self.body(st.batch, st.target, self.ws, self.bce, self.z, self.dz, pre=pre)
        else:
            st.copy_in(k)
            self.body(st.batch, st.target, self.ws, self.bce, self.z, self.dz)

    def __call__(self, plan: HostPlan, target: np.ndarray):
        k = self.calls % StaticBatch.SLOTS
        self.calls += 1
        if self.done[k] is not None:
            self.done[k].synchronize()
        self.static.fill(plan, target, k)
        cur = torch.cuda.current_stream(self.device)
        if self.graphs[k] is not None:
            self.graphs[k].replay()
            self.replays += 1
        else:
            self._issue(k)
            if self.use_graph:
                # capture on torch's side stream; the eager step above already sized every buffer.
                # Every slot's graph now: a capture issues nothing, so the next call already replays
                cur.synchronize()
                for j in range(StaticBatch.SLOTS):
                    g = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(g):
                        self._issue(j)
                    self.graphs[j] = g
        if self.done[k] is None:
            self.done[k] = SlotEvent()
        self.done[k].record(cur)


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
