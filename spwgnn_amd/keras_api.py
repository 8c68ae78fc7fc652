"""Keras-shaped front end: PropagationNetwork.getModel(...) → model.fit / model.predict.

Mirrors the reference call sites one-to-one so a driver written against the reference drops in:
  * PropagationNetwork().getModel(n_objects, object_dim=3, relation_dim=1)  — Networks.py:12-104
    (one model per n_objects, cached at Networks.py:17-18,103; all models share rm/om/rmp/omp weights, :40-56)
  * model.fit(x_dict, {'target': y}, batch_size=32, epochs=10, validation_split=0.2, shuffle=True,
    verbose=1)                                                            — main.py:92-98
  * model.predict(x_dict) → (B, N, 1) probabilities                       — JengaBuilder.py:328-329
Compile semantics (Networks.py:101-102): Adam(lr=5e-4, decay=0) per model, binary_crossentropy,
binary_accuracy. Every step runs through libspwgnn_hip (forward, BCE, backward, Adam).
"""
from __future__ import annotations

from typing import Dict, List, Optional

import numpy as np
import torch

from . import _lib
from . import engine as E
from . import params as P
from .batch import HostPlan, TowerBatch
from .network import GraphNetwork
from .replay import DeviceCounters, ReplayCache


class CompactDataset:
    """Host-side compact copy of a dense dataset: per-tower node rows and active edges."""

    def __init__(self, objects, Rs, Rr, propagation=None):
        objects = np.asarray(objects, np.float32)
        self.B, self.N = objects.shape[:2]
        full = TowerBatch.from_dense(objects[:1], np.asarray(Rs)[:1], np.asarray(Rr)[:1], device="cpu")  # validates layout
        del full
        # one C++ conversion for the whole set
        import ctypes as C
        from . import _lib
        Rs = np.ascontiguousarray(Rs, np.float32)
        Rr = np.ascontiguousarray(Rr, np.float32)
        E_ = self.N * (self.N - 1)
        cap = self.B * E_
        src = np.zeros(max(cap, 1), np.int32)
        dst = np.zeros(max(cap, 1), np.int32)
        tec = np.zeros(self.B, np.int32)
        ne = C.c_int64(0)
        _lib.check(_lib.lib().spwgnn_dense_to_edges(Rs.ctypes.data, Rr.ctypes.data, self.B, self.N, src.ctypes.data,
                                                    dst.ctypes.data, None, cap, C.byref(ne), tec.ctypes.data),
                   "dense_to_edges")
        n = int(ne.value)
        self.objects = objects
        self.src = src[:n] - np.repeat(np.arange(self.B, dtype=np.int32) * self.N, tec)   # tower-local
        self.dst = dst[:n] - np.repeat(np.arange(self.B, dtype=np.int32) * self.N, tec)
        self.edge_off = np.concatenate([[0], np.cumsum(tec)]).astype(np.int64)
        self.tower_edges = tec
        self.prop = None if propagation is None or not np.any(np.asarray(propagation)) else \
            np.asarray(propagation, np.float32)

    def subset(self, idx: np.ndarray, device) -> TowerBatch:
        return TowerBatch.from_plan(self.subset_plan(idx), device)

    def subset_plan(self, idx: np.ndarray, edge_cap: bool = False) -> HostPlan:
        """Host plan of the towers `idx`; `edge_cap`: blocks sized for all N(N−1) relation slots
        per tower, so every batch of len(idx) towers has one geometry (replayed steps)."""
        idx = np.asarray(idx)
        n = len(idx)
        # the towers' edge ranges gathered in one vectorised pass (tower k of the batch: node ids + k·N)
        cnt = self.tower_edges[idx].astype(np.int64)
        tot = int(cnt.sum())
        first = np.cumsum(cnt) - cnt                         # batch position of each tower's first edge
        gidx = np.arange(tot, dtype=np.int64) + np.repeat(self.edge_off[idx] - first, cnt)
        shift = np.repeat(np.arange(n, dtype=np.int32) * self.N, cnt)
        src = (self.src[gidx] + shift).astype(np.int32)
        dst = (self.dst[gidx] + shift).astype(np.int32)
        prop = None if self.prop is None else self.prop[idx].reshape(n * self.N, 100)
        return HostPlan.build(self.objects[idx].reshape(n * self.N, 3), np.full(n, self.N, np.int32), src, dst,
                              self.tower_edges[idx], prop, node_shape=(n, self.N),
                              edge_cap=self.N * (self.N - 1) if edge_cap else None)


class KerasModel:
    """One compiled per-N model of the reference (Networks.py:99-104); weights shared via ``net``."""

    def __init__(self, net: GraphNetwork, n_objects: int, object_dim: int = 3, lr: float = 5e-4,
                 l2: float = 0.0):
        if object_dim != 3:
            # Networks.py:70-73 + main.py:28-31/59-63: the object_dim=2 path of the reference is
            # broken (om gets 1 feature, boxes[...,2] is out of range); only the Jenga layout runs.
            raise ValueError("only object_dim=3 ([x, y, width]) is supported, as in the working reference path")
        self.net = net
        self.n_objects = n_objects
        self.lr, self.l2 = lr, l2
        self.beta1, self.beta2, self.eps = 0.9, 0.999, 1e-7
        dev = net.device
        self.m = torch.zeros_like(net.flat.data)
        self.v = torch.zeros_like(net.flat.data)
        self.iterations = 0
        self._ws = E.Workspace(dev)
        self._bce = E.BceScratch(dev)
        self._grads = torch.empty_like(net.flat.data)
        self.history: Dict[str, List[float]] = {}
        # replayed fit steps (spwgnn_amd/replay.py): device step words, per-geometry graphs, epoch sums
        self._ctr: Optional[DeviceCounters] = None
        self._replays: Optional[ReplayCache] = None
        self._replay_graph: Optional[bool] = None
        self._tot = torch.zeros(3, dtype=torch.float64, device=dev)
        self._w3: Dict[int, torch.Tensor] = {}

    # ---------------------------------------------------------------- inference
    def predict(self, x: Dict[str, np.ndarray], batch_size: int = 32768) -> np.ndarray:
        objects = np.asarray(x["objects"], np.float32)
        B, N = objects.shape[:2]
        out = np.zeros((B, N, 1), np.float32)
        run = E.RunConfig(self.net.mp_steps, training=False)
        for b0 in range(0, B, batch_size):
            sl = slice(b0, min(B, b0 + batch_size))
            prop = x.get("propagation")
            batch = TowerBatch.from_dense(objects[sl], np.asarray(x["sender_relations"])[sl],
                                          np.asarray(x["receiver_relations"])[sl],
                                          None if prop is None else np.asarray(prop)[sl], device=self.net.device)
            with torch.no_grad():
                z = E.forward(self.net.flat.detach(), batch, run, self._ws)
                p = E.sigmoid(z)
            out[sl, :, 0] = p.reshape(-1, N).cpu().numpy()
        return out

    # ---------------------------------------------------------------- training
    def train_on_batch(self, batch: TowerBatch, target: torch.Tensor):
        """One Keras step: forward (dropout on), BCE, backward, Adam. Returns (loss, accuracy) tensors."""
        net = self.net
        net._step_seed += 1
        run = E.RunConfig(net.mp_steps, training=True, dropout=net.dropout, seed=net._step_seed)
        z = E.forward(net.flat.data, batch, run, self._ws)
        out3, dz = E.bce(z, target, self._bce)
        E.backward(net.flat.data, batch, run, self._ws, dz, grads=self._grads)
        self.iterations += 1
        E.adam(net.flat.data, self._grads, self.m, self.v, self.iterations, self.lr, self.beta1, self.beta2,
               self.eps, self.l2)
        return out3

    def _replay_body(self):
        """One fit step's launches for a replayed geometry: the same sequence as train_on_batch
        (key + 1, forward, BCE, backward, Adam at the incremented step) with the per-step scalars
        read from the device, and the epoch sums accumulated on the device."""
        net, ctr = self.net, self._ctr

        def body(batch, target, ws, bce, z, dz, pre=None):
            w3 = self._w3[batch.n_towers]        # created before the first (eager) run of a geometry
            # the key/step advance (and the replayed batch upload, `pre`) ride in the forward's first launch
            pro = None
            if E.FOLD_PROLOGUE:
                pro = pre if pre is not None else E.Prologue()
                pro.key, pro.step, pro.mode = ctr.key, ctr.step, _lib.STEP_KEY_COUNTER
            else:
                E.step_advance(ctr.key, ctr.step, _lib.STEP_KEY_COUNTER)
            run = E.RunConfig(net.mp_steps, training=True, dropout=net.dropout, seed_dev=ctr.key, prologue=pro)
            E.forward(net.flat.data, batch, run, ws, logits=z)
            # loss + epoch sums and the backward in one call: on the fused small-batch loop the loss
            # needs no launch of its own (spwgnn_bce_backward)
            E.bce_backward(net.flat.data, batch, run, ws, z, target, bce, dlogits=dz, total3=self._tot, weights3=w3,
                           grads=self._grads)
            E.adam_dev(net.flat.data, self._grads, self.m, self.v, ctr.step, ctr.lr_table, self.beta1, self.beta2,
                       self.eps, self.l2)
        return body

    def evaluate_batch(self, batch: TowerBatch, target: torch.Tensor):
        run = E.RunConfig(self.net.mp_steps, training=False)
        z = E.forward(self.net.flat.data, batch, run, self._ws)
        out3, _ = E.bce(z, target, self._bce)
        return out3

    def fit(self, x: Dict[str, np.ndarray], y: Dict[str, np.ndarray], batch_size: int = 32, epochs: int = 10,
            validation_split: float = 0.0, shuffle: bool = True, verbose: int = 1, seed: int = 0,
            graph: bool = False):
        """Keras fit (main.py:92-98). Each training step is the replayable step of
        spwgnn_amd/replay.py — forward, BCE, backward and Adam per batch geometry on static buffers
        refilled by the step's first launch — issued eagerly (`graph=True`: the same step captured
        once and replayed as a hipGraph; bit-identical results; on the MI355X host eager issue is the
        faster, 0.270 vs 0.277 ms per step at batch 32); batches are planned with
        N(N−1) relation slots per tower."""
        objects = np.asarray(x["objects"], np.float32)
        target = np.asarray(y["target"], np.float32).reshape(objects.shape[0], -1)
        B = objects.shape[0]
        n_tr = keras_split_at(B, validation_split)
        n_val = B - n_tr
        ds = CompactDataset(objects, x["sender_relations"], x["receiver_relations"], x.get("propagation"))
        rng = np.random.default_rng(seed)
        dev = self.net.device
        hist = {"loss": [], "binary_accuracy": []}
        if n_val:
            hist.update({"val_loss": [], "val_binary_accuracy": []})
            vbatch = ds.subset(np.arange(n_tr, B), dev)
            vtgt = torch.as_tensor(target[n_tr:], device=dev).reshape(-1).contiguous()
        # every step runs as a replayed hipGraph per batch geometry (graph=False: the same launches
        # eagerly); the device words start from the host counters and the host mirrors each step
        if self._ctr is None:
            self._ctr = DeviceCounters(dev, self.net._step_seed, self.iterations, self.lr, self.beta1,
                                       self.beta2)
        else:
            self._ctr.set(key=self.net._step_seed, step=self.iterations, lr=self.lr, beta1=self.beta1,
                          beta2=self.beta2)
        if self._replays is None or self._replay_graph != graph:
            self._replays = ReplayCache(dev, self._replay_body, graph=graph)
            self._replay_graph = graph
        # per-epoch sums stay on the device (stream-ordered copies) and are read once after the last
        # epoch — with verbose=0 the host never waits for the GPU between epochs (a sync per epoch
        # drained the pipeline: ≈ 8 µs per step at batch 32); verbose > 0 reads them per epoch to print
        ep_tot = torch.zeros(epochs, 3, dtype=torch.float64, device=dev)
        ep_val = torch.zeros(epochs, 3, dtype=torch.float32, device=dev)

        def record(ep):
            tot_l, tot_c, tot_n = ep_tot[ep].tolist()
            hist["loss"].append(tot_l / max(n_tr, 1))
            hist["binary_accuracy"].append(tot_c / max(tot_n, 1))
            if n_val:
                vl, vc, vn = ep_val[ep].tolist()
                hist["val_loss"].append(vl)
                hist["val_binary_accuracy"].append(vc / vn)

        for ep in range(epochs):
            order = rng.permutation(n_tr) if shuffle else np.arange(n_tr)
            # (Σ loss·batch, Σ correct, Σ nodes) on the device: no host sync per batch, so the host
            # builds the next batch while the GPU runs this one
            self._tot.zero_()
            for b0 in range(0, n_tr, batch_size):
                idx = order[b0:b0 + batch_size]
                if len(idx) not in self._w3:
                    self._w3[len(idx)] = torch.tensor([float(len(idx)), 1.0, 1.0], dtype=torch.float64, device=dev)
                self._replays(ds.subset_plan(idx, edge_cap=True), target[idx])
                self.net._step_seed += 1
                self.iterations += 1
            ep_tot[ep].copy_(self._tot)
            if n_val:
                ep_val[ep].copy_(self.evaluate_batch(vbatch, vtgt))
            if verbose:
                record(ep)
                msg = f"Epoch {ep + 1}/{epochs} - loss: {hist['loss'][-1]:.4f} - binary_accuracy: {hist['binary_accuracy'][-1]:.4f}"
                if n_val:
                    msg += f" - val_loss: {hist['val_loss'][-1]:.4f} - val_binary_accuracy: {hist['val_binary_accuracy'][-1]:.4f}"
                print(msg)
        if not verbose:
            for ep in range(epochs):
                record(ep)
        for k, v in hist.items():
            self.history.setdefault(k, []).extend(v)
        return hist


def keras_split_at(n_samples: int, validation_split: float) -> int:
    """Number of training samples Keras 2.x keeps for fit(validation_split=v) (main.py:96):
    split_at = int(n · (1 − v)); the validation set is the LAST n − split_at samples, taken before
    shuffling."""
    if not validation_split:
        return int(n_samples)
    if not 0.0 < validation_split < 1.0:
        raise ValueError("validation_split must be in [0, 1)")
    return int(int(n_samples) * (1.0 - validation_split))


class PropagationNetwork:
    """Networks.py:12-104: getModel caches one compiled model per n_objects, all sharing the
    weights of the first one built (set_weights / reuse_model, Networks.py:40-56)."""

    def __init__(self, device="cuda", seed: int = 0, mp_steps: int = E.REF_MP_STEPS, dropout: float = E.REF_DROPOUT):
        self.Nets: Dict[int, KerasModel] = {}
        self.set_weights = False
        self._net: Optional[GraphNetwork] = None
        self._device, self._seed, self._mp, self._drop = device, seed, mp_steps, dropout

    def getModel(self, n_objects: int, object_dim: int = 3, relation_dim: int = 1) -> KerasModel:  # noqa: N802
        if n_objects in self.Nets:
            return self.Nets[n_objects]
        if not self.set_weights:
            self._net = GraphNetwork(self._mp, self._drop, self._seed, device=self._device)
            self.set_weights = True
        model = KerasModel(self._net, n_objects, object_dim)
        self.Nets[n_objects] = model
        return model
