"""TowerBatch: the reference's 4-tensor input dict, compacted for the HIP kernels.

The reference feeds Keras (B, N, 3) objects, two dense (B, N, E) one-hot relation matrices and a
(B, N, 100) propagation state (src/Networks.py:22-29; built by src/main.py:66-93). Every active
relation column is one sender and one receiver, so the batch becomes a union graph: node rows
(objects, propagation) and an edge list, packed by the C library into wave-tiles of whole towers
and 32-edge blocks (spwgnn_plan_size/fill). Conversion happens once per batch on the host (C++);
the device arrays then stay resident in HBM.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field
from typing import Optional

import numpy as np
import torch

from . import _lib


def _ptr(a: np.ndarray) -> int:
    return a.ctypes.data


SMALL_BATCH_TOWERS = 2048   # below this a batch cannot fill the chip's 2,048 edge waves anyway


def default_nw_max(max_nodes: int, n_towers: int = 1 << 30) -> int:
    """Nodes per wave-tile: at least one whole tower. Up to 16 nodes the backward segment sums run
    as one one-hot matrix product (receiver rows 0-15, sender rows 16-31), so small towers are
    packed up to 16 nodes per wave; larger towers take one wave-tile each (≤ 32 nodes). A small
    batch (fewer towers than the edge kernels have waves) takes one tower per wave-tile instead:
    each wave then walks one tower's blocks, not two or three, which is the step's latency at
    batch 32 (the reference's fit, main.py:92-98)."""
    if max_nodes > 16:
        return int(min(_NW_LIMIT, max_nodes))
    return max(int(max_nodes), 1) if n_towers < SMALL_BATCH_TOWERS else 16


_NW_LIMIT = 32


def upload(arrays, device) -> list:
    """Host arrays → device tensors in ONE copy: packed (16-byte aligned) into a pinned staging
    buffer and copied with non_blocking=True, so the host does not wait for the stream to drain (a
    copy from pageable memory does) and can build the next batch while the GPU runs this one. The
    caching host allocator keeps the staging block until its copy has run."""
    dev = torch.device(device)
    arrays = [np.ascontiguousarray(a) for a in arrays]
    if dev.type != "cuda":
        return [torch.from_numpy(a.copy()) for a in arrays]
    offs, total = [], 0
    for a in arrays:
        offs.append(total)
        total += (a.nbytes + 15) // 16 * 16
    host = torch.empty(max(total, 16), dtype=torch.uint8, pin_memory=True)
    hv = host.numpy()
    for a, o in zip(arrays, offs):
        hv[o:o + a.nbytes] = a.reshape(-1).view(np.uint8)
    d = host.to(dev, non_blocking=True)
    out = []
    for a, o in zip(arrays, offs):
        t = d[o:o + a.nbytes].view(torch.from_numpy(a[:0].reshape(-1)).dtype) if a.nbytes else \
            torch.empty(0, dtype=torch.from_numpy(a[:0].reshape(-1)).dtype, device=dev)
        out.append(t.view(a.shape))
    return out


def pack_order(tower_nodes, tower_edges, nw_max: int = 16) -> np.ndarray:
    """spwgnn_plan_order: a tower order that packs a ragged batch into fewer 32-edge blocks (towers by
    decreasing edge count into the wave-tile whose last block has room; include/spwgnn.h)."""
    tn = np.ascontiguousarray(tower_nodes, dtype=np.int32)
    te = np.ascontiguousarray(tower_edges, dtype=np.int32)
    order = np.zeros(len(tn), np.int32)
    if len(tn):
        _lib.check(_lib.lib().spwgnn_plan_order(len(tn), _ptr(tn), _ptr(te), int(nw_max), _ptr(order)), "plan_order")
    return order


def reorder_towers(pos, tower_nodes, src, dst, tower_edges, order, prop=None):
    """The towers of a compact edge-form batch in `order` (order[k] = the k-th tower): node rows,
    edges (node ids rebased), counts. Returns (pos, tower_nodes, src, dst, tower_edges, prop, node_perm)
    with node_perm[i] = the input-order index of node i of the reordered batch."""
    tn = np.asarray(tower_nodes, np.int64)
    te = np.asarray(tower_edges, np.int64)
    order = np.asarray(order, np.int64)
    noff = np.concatenate([[0], np.cumsum(tn)])
    eoff = np.concatenate([[0], np.cumsum(te)])
    node_perm = np.concatenate([np.arange(noff[t], noff[t + 1]) for t in order]) if len(order) else np.zeros(0, np.int64)
    edge_perm = np.concatenate([np.arange(eoff[t], eoff[t + 1]) for t in order]) if len(order) else np.zeros(0, np.int64)
    new_noff = np.concatenate([[0], np.cumsum(tn[order])])
    shift = np.repeat(new_noff[:-1] - noff[order], te[order])     # per reordered edge: old → new node base
    src = np.asarray(src, np.int64)[edge_perm] + shift
    dst = np.asarray(dst, np.int64)[edge_perm] + shift
    pos = np.asarray(pos)[node_perm]
    prop = None if prop is None else np.asarray(prop).reshape(int(noff[-1]), -1)[node_perm]
    return (pos, tn[order].astype(np.int32), src.astype(np.int32), dst.astype(np.int32), te[order].astype(np.int32),
            prop, node_perm)


@dataclass
class HostPlan:
    """A batch's host-side arrays in upload order (pos4, node_tower, node_local, wtile, edge_src,
    edge_dst, blk_csr[, prop]) plus the sizes the kernels are launched with."""
    n_towers: int
    n_nodes: int
    tower_nodes: np.ndarray
    tower_edges: np.ndarray
    src: np.ndarray
    dst: np.ndarray
    n_wtiles: int
    n_eblocks: int
    nw_max: int
    edge_id: np.ndarray
    node_shape: Optional[tuple]
    has_prop: bool
    arrays: list
    flags: int = 0     # spwgnn_batch.flags (_lib.BATCH_RECV_BLOCKS: a receiver-block plan)
    node_perm: Optional[np.ndarray] = None   # packed plans: node i of the plan = input node node_perm[i]

    @property
    def geometry(self) -> tuple:
        """What a captured step bakes in: sizes, layout flags and every array's shape."""
        return (self.n_towers, self.n_nodes, self.n_wtiles, self.n_eblocks, self.nw_max, self.has_prop, self.flags,
                tuple(a.shape for a in self.arrays))

    @staticmethod
    def build(pos, tower_nodes, src, dst, tower_edges, prop=None, nw_max=None, node_shape=None, tower_ids=None,
              edge_cap=None, recv_blocks=None, pack: bool = False) -> "HostPlan":
        """recv_blocks: one 32-edge block per node holding its in-edges (spwgnn_plan_fill_recv; the x6
        edge forward then sums a node's messages as a column sum). None = automatic: for wave-tiles of
        more than 16 nodes whose blocks would be ≥ 80 % full (large, densely connected towers —
        BASELINE config 5), never with edge_cap.
        pack: plan the towers in spwgnn_plan_order's order (ragged batches: fewer, fuller blocks). Each
        tower keeps its id (dropout key) and `node_perm` maps the plan's node rows back to the input's:
        logits and d/d'propagation' come out in plan order (TowerBatch.to_input_order), targets go in
        in plan order (TowerBatch.to_plan_order)."""
        if pack:
            tn0 = np.asarray(tower_nodes, np.int32)
            if nw_max is None:
                nw_max = default_nw_max(int(tn0.max()) if len(tn0) else 1, len(tn0))
            order = pack_order(tn0, tower_edges, min(int(nw_max), 16) if int(tn0.max()) <= 16 else int(nw_max))
            tid0 = np.arange(len(tn0), dtype=np.int64) if tower_ids is None else np.asarray(tower_ids, np.int64)
            pos, tower_nodes, src, dst, tower_edges, prop, perm = reorder_towers(pos, tn0, src, dst, tower_edges, order,
                                                                                prop)
            cap = None if edge_cap is None else np.broadcast_to(np.asarray(edge_cap, np.int32), (len(tn0),))[order]
            plan = HostPlan.build(pos, tower_nodes, src, dst, tower_edges, prop, nw_max, None, tid0[order], cap,
                                  recv_blocks)
            plan.node_perm = perm
            return plan
        L = _lib.lib()
        tower_nodes = np.ascontiguousarray(tower_nodes, dtype=np.int32)
        tower_edges = np.ascontiguousarray(tower_edges, dtype=np.int32)
        src = np.ascontiguousarray(src, dtype=np.int32)
        dst = np.ascontiguousarray(dst, dtype=np.int32)
        T = len(tower_nodes)
        Nn = int(tower_nodes.sum())
        if T == 0:
            raise ValueError("empty batch: at least one tower is needed")
        if pos.shape[0] != Nn:
            raise ValueError(f"pos has {pos.shape[0]} rows, towers hold {Nn} nodes")
        if int(tower_edges.sum()) != len(src) or len(src) != len(dst):
            raise ValueError("edge counts do not match the edge list")
        if nw_max is None:
            nw_max = default_nw_max(int(tower_nodes.max()) if T else 1, T)
        if T and int(tower_nodes.max()) > _NW_LIMIT:
            raise ValueError(f"towers of more than {_NW_LIMIT} nodes are not supported by this build")
        if recv_blocks is None:
            recv_blocks = (edge_cap is None and nw_max > 16 and len(src) > 0 and Nn * 32 <= 1.25 * len(src)
                           and int(np.bincount(dst, minlength=Nn).max()) <= 32)
        if recv_blocks and edge_cap is not None:
            raise ValueError("receiver-block plans do not take edge capacities")
        cap = None
        if edge_cap is not None:
            cap = np.ascontiguousarray(np.broadcast_to(np.asarray(edge_cap, np.int32), (T,)), dtype=np.int32)
            if np.any(cap < tower_edges):
                raise ValueError("edge_cap must be >= every tower's edge count")
        sizes = _lib.PlanSizes()
        if recv_blocks:
            _lib.check(L.spwgnn_plan_size_recv(T, _ptr(tower_nodes), nw_max, C.byref(sizes)), "plan_size_recv")
        elif cap is None:
            _lib.check(L.spwgnn_plan_size(T, _ptr(tower_nodes), _ptr(tower_edges), nw_max, C.byref(sizes)), "plan_size")
        else:
            _lib.check(L.spwgnn_plan_size_cap(T, _ptr(tower_nodes), _ptr(cap), nw_max, C.byref(sizes)), "plan_size_cap")
        wtile = np.zeros((sizes.n_wtiles, 4), np.int32)
        esrc = np.zeros(sizes.n_eblocks * 32, np.int32)
        edst = np.zeros(sizes.n_eblocks * 32, np.int32)
        eid = np.zeros(sizes.n_eblocks * 32, np.int32)
        csr = np.zeros((sizes.n_eblocks, 128), np.uint8)
        sp = _ptr(src) if len(src) else None
        dp = _ptr(dst) if len(dst) else None
        if recv_blocks:
            _lib.check(L.spwgnn_plan_fill_recv(T, _ptr(tower_nodes), _ptr(tower_edges), sp, dp, nw_max, C.byref(sizes),
                                               _ptr(wtile), _ptr(esrc), _ptr(edst), _ptr(eid), _ptr(csr)), "plan_fill_recv")
        elif cap is None:
            _lib.check(L.spwgnn_plan_fill(T, _ptr(tower_nodes), _ptr(tower_edges), sp, dp, nw_max, C.byref(sizes),
                                          _ptr(wtile), _ptr(esrc), _ptr(edst), _ptr(eid), _ptr(csr)), "plan_fill")
        else:
            _lib.check(L.spwgnn_plan_fill_cap(T, _ptr(tower_nodes), _ptr(tower_edges), _ptr(cap), sp, dp, nw_max,
                                              C.byref(sizes), _ptr(wtile), _ptr(esrc), _ptr(edst), _ptr(eid),
                                              _ptr(csr)), "plan_fill_cap")
        tid = np.arange(T, dtype=np.int32) if tower_ids is None else np.asarray(tower_ids, np.int64)
        if len(tid) != T or (T and (tid.min() < 0 or tid.max() > np.iinfo(np.int32).max)):
            raise ValueError("tower_ids must hold one non-negative int32 id per tower")
        node_tower = np.repeat(tid.astype(np.int32), tower_nodes)
        starts = np.concatenate([[0], np.cumsum(tower_nodes)[:-1]]).astype(np.int64)
        node_local = (np.arange(Nn) - np.repeat(starts, tower_nodes)).astype(np.int32)
        pos4 = np.zeros((Nn, 4), np.float32)
        pos4[:, :3] = np.asarray(pos, np.float32)[:, :3]
        host = [pos4, node_tower, node_local, wtile, esrc, edst, csr]
        if prop is not None:
            host.append(np.asarray(prop, np.float32).reshape(Nn, 100))
        return HostPlan(T, Nn, tower_nodes, tower_edges, src, dst, sizes.n_wtiles, sizes.n_eblocks, sizes.nw_max,
                        eid, node_shape, prop is not None, host, _lib.BATCH_RECV_BLOCKS if recv_blocks else 0)


@dataclass
class TowerBatch:
    n_towers: int
    n_nodes: int
    tower_nodes: np.ndarray          # (T,) int32
    tower_edges: np.ndarray          # (T,) int32 active relations per tower
    src: np.ndarray                  # (Ne,) int32 global sender (host copy)
    dst: np.ndarray                  # (Ne,) int32 global receiver
    n_wtiles: int
    n_eblocks: int
    nw_max: int
    device: torch.device
    pos: torch.Tensor                # (Nn, 4) f32
    prop: Optional[torch.Tensor]     # (Nn, 100) f32 or None (= zeros)
    node_tower: torch.Tensor
    node_local: torch.Tensor
    wtile: torch.Tensor
    edge_src: torch.Tensor
    edge_dst: torch.Tensor
    blk_csr: torch.Tensor
    edge_id: np.ndarray              # (n_eblocks*32,) original edge index or -1
    node_shape: Optional[tuple] = None   # (B, N) when built from a uniform-N dense batch
    flags: int = 0                       # spwgnn_batch.flags (the plan's layout)
    node_perm: Optional[np.ndarray] = None   # packed plans (HostPlan.build pack=True): plan node i = input node node_perm[i]
    _cstruct: Optional[_lib.BatchC] = field(default=None, repr=False)

    def to_plan_order(self, x):
        """Per-node rows (targets, propagation) in the input's node order → the plan's (identity
        unless the plan was packed). numpy or torch, first axis = nodes."""
        if self.node_perm is None:
            return x
        if isinstance(x, torch.Tensor):
            return x[torch.as_tensor(self.node_perm, device=x.device)]
        return np.asarray(x)[self.node_perm]

    def to_input_order(self, x):
        """Per-node results (logits, d/d'propagation') in the plan's node order → the input's."""
        if self.node_perm is None:
            return x
        if isinstance(x, torch.Tensor):
            out = torch.empty_like(x)
            out[torch.as_tensor(self.node_perm, device=x.device)] = x
            return out
        out = np.empty_like(np.asarray(x))
        out[self.node_perm] = x
        return out

    @property
    def n_edges(self) -> int:
        return int(len(self.src))

    @property
    def tower_offsets(self) -> torch.Tensor:
        """(T+1,) int32 device node offsets of the towers (built on first use)."""
        t = getattr(self, "_tower_offsets", None)
        if t is None:
            off = np.concatenate([[0], np.cumsum(self.tower_nodes)]).astype(np.int32)
            t = torch.from_numpy(off).to(self.device)
            object.__setattr__(self, "_tower_offsets", t)
        return t

    # ------------------------------------------------------------------ constructors
    @staticmethod
    def from_edges(pos: np.ndarray, tower_nodes, src, dst, tower_edges, prop=None, device="cuda",
                   nw_max: Optional[int] = None, node_shape=None, tower_ids=None, edge_cap=None,
                   recv_blocks=None, pack: bool = False) -> "TowerBatch":
        """pos (Nn, >=3) objects rows (already /170); towers are consecutive node ranges;
        edges tower-major with global node ids. `tower_ids` (T,): each tower's index in the batch it
        was cut from (the dropout masks are keyed by it), so a shard or micro-batch of a larger batch
        draws the masks the whole batch would; default 0..T-1. `edge_cap` (T,) ≥ tower_edges: size
        each tower's blocks for that many edges (spwgnn_plan_fill_cap) so same-shape batches share
        one plan geometry (replayed hipGraph steps); default: the actual edge counts."""
        plan = HostPlan.build(pos, tower_nodes, src, dst, tower_edges, prop, nw_max, node_shape, tower_ids, edge_cap,
                              recv_blocks, pack)
        return TowerBatch.from_plan(plan, device)

    @staticmethod
    def from_plan(plan: "HostPlan", device, dev_arrays: Optional[list] = None) -> "TowerBatch":
        """A device batch from a host plan: its arrays uploaded in one copy, or `dev_arrays` (device
        tensors of the plan's array shapes, e.g. a replayed step's static buffers) used as they are."""
        dev = torch.device(device)
        d = dev_arrays if dev_arrays is not None else upload(plan.arrays, dev)
        m = plan
        prop_t = d[7] if m.has_prop else None
        return TowerBatch(m.n_towers, m.n_nodes, m.tower_nodes, m.tower_edges, m.src, m.dst, m.n_wtiles, m.n_eblocks,
                          m.nw_max, dev, d[0], prop_t, d[1], d[2], d[3], d[4], d[5], d[6], m.edge_id, m.node_shape,
                          m.flags, m.node_perm)

    @staticmethod
    def from_dense(objects, sender_relations, receiver_relations, propagation=None, device="cuda",
                   nw_max: Optional[int] = None) -> "TowerBatch":
        """The reference input dict (Networks.py:22-29) → compact batch (C++ conversion)."""
        to_np = lambda x: x.detach().cpu().numpy() if isinstance(x, torch.Tensor) else np.asarray(x)
        obj = np.ascontiguousarray(to_np(objects), np.float32)
        Rs = np.ascontiguousarray(to_np(sender_relations), np.float32)
        Rr = np.ascontiguousarray(to_np(receiver_relations), np.float32)
        B, N = obj.shape[:2]
        E = N * (N - 1)
        if Rs.shape != (B, N, E) or Rr.shape != (B, N, E):
            raise ValueError(f"relation matrices must be (B, N, N(N-1)) = {(B, N, E)}; got {Rs.shape}, {Rr.shape}")
        L = _lib.lib()
        cap = B * E
        src = np.zeros(max(cap, 1), np.int32)
        dst = np.zeros(max(cap, 1), np.int32)
        tec = np.zeros(B, np.int32)
        ne = C.c_int64(0)
        _lib.check(L.spwgnn_dense_to_edges(_ptr(Rs), _ptr(Rr), B, N, _ptr(src), _ptr(dst), None, cap, C.byref(ne),
                                           _ptr(tec)), "dense_to_edges")
        n = int(ne.value)
        prop = None
        if propagation is not None:
            p = to_np(propagation)
            if np.any(p != 0):
                prop = np.asarray(p, np.float32).reshape(B * N, 100)
        return TowerBatch.from_edges(obj.reshape(B * N, 3), np.full(B, N, np.int32), src[:n], dst[:n], tec, prop,
                                     device, nw_max, node_shape=(B, N))

    @staticmethod
    def fully_connected(objects: np.ndarray, propagation=None, device="cuda", nw_max=None,
                        tower_ids=None, recv_blocks=None) -> "TowerBatch":
        """Fast path for (B, N, 3) towers whose relations are all active (the inference relation
        set of JengaBuilder.py:309-326 and the benchmark configs)."""
        obj = np.asarray(objects, np.float32)
        B, N = obj.shape[:2]
        m_idx, j_idx = np.nonzero(~np.eye(N, dtype=bool))
        base = (np.arange(B, dtype=np.int64) * N)[:, None]
        src = (base + m_idx[None, :]).reshape(-1).astype(np.int32)
        dst = (base + j_idx[None, :]).reshape(-1).astype(np.int32)
        prop = None if propagation is None else np.asarray(propagation, np.float32).reshape(B * N, 100)
        return TowerBatch.from_edges(obj.reshape(B * N, 3), np.full(B, N, np.int32), src, dst,
                                     np.full(B, N * (N - 1), np.int32), prop, device, nw_max, node_shape=(B, N),
                                     tower_ids=tower_ids, recv_blocks=recv_blocks)

    @staticmethod
    def ragged(objects_list, relation_threshold: Optional[float] = None, device="cuda", nw_max=None,
               raw_positions_list=None) -> "TowerBatch":
        """Towers of different sizes: list of (N_b, 3) objects; relations fully connected, or
        thresholded on ``raw_positions_list`` (pixels) like main.py:71-81."""
        if len(objects_list) == 0:
            raise ValueError("empty batch: at least one tower is needed")
        tower_nodes = np.array([len(o) for o in objects_list], np.int32)
        srcs, dsts, tes = [], [], []
        off = 0
        for b, o in enumerate(objects_list):
            N = len(o)
            m_idx, j_idx = np.nonzero(~np.eye(N, dtype=bool))
            if relation_threshold is not None:
                raw = np.asarray(raw_positions_list[b])
                keep = np.linalg.norm(raw[m_idx, 0:2] - raw[j_idx, 0:2], axis=1) < relation_threshold
                m_idx, j_idx = m_idx[keep], j_idx[keep]
            srcs.append(off + m_idx)
            dsts.append(off + j_idx)
            tes.append(len(m_idx))
            off += N
        src = np.concatenate(srcs).astype(np.int32) if srcs else np.zeros(0, np.int32)
        dst = np.concatenate(dsts).astype(np.int32) if dsts else np.zeros(0, np.int32)
        pos = np.concatenate([np.asarray(o, np.float32) for o in objects_list], axis=0)
        return TowerBatch.from_edges(pos, tower_nodes, src, dst, np.array(tes, np.int32), None, device, nw_max)

    # ------------------------------------------------------------------ C view
    def cstruct(self) -> _lib.BatchC:
        if self._cstruct is None:
            b = _lib.BatchC()
            b.n_towers, b.n_nodes = self.n_towers, self.n_nodes
            b.n_wtiles, b.n_eblocks, b.nw_max = self.n_wtiles, self.n_eblocks, self.nw_max
            b.flags = self.flags
            b.pos = self.pos.data_ptr()
            b.prop = self.prop.data_ptr() if self.prop is not None else None
            b.node_tower = self.node_tower.data_ptr()
            b.node_local = self.node_local.data_ptr()
            b.wtile = self.wtile.data_ptr()
            b.edge_src = self.edge_src.data_ptr()
            b.edge_dst = self.edge_dst.data_ptr()
            b.blk_csr = self.blk_csr.data_ptr()
            self._cstruct = b
        return self._cstruct

    def with_prop(self, prop: Optional[torch.Tensor]) -> "TowerBatch":
        """Same graph, different propagation input (device tensor (Nn, 100) or None)."""
        nb = TowerBatch(**{k: getattr(self, k) for k in self.__dataclass_fields__ if k != "_cstruct"})
        nb.prop = None if prop is None else prop.reshape(self.n_nodes, 100).to(self.device, torch.float32).contiguous()
        return nb
