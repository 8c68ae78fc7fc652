"""Batched simulator-side inference and the optional per-tower pooling (row 4).

The reference asks the GNN one B=1 `predict` per candidate:
  * `JengaBuilder.remove_to_demolish` (JengaBuilder.py:236-259): for every box i, the tower with box i
    removed → Σ_objects ŷ; the box whose removal gives the smallest sum is removed;
  * `TowerCreator.drop_to_demolish` (TowerCreator.py:276-307): 100 candidate drop positions →
    Σ ŷ each → argmin.
Here all candidates of a decision form ONE batch: one forward over the candidate towers, the
per-tower Σ sigmoid(z) on device (`spwgnn_tower_readout`), and the argmin.

Inference relations are built exactly as the reference's `predict_stabilities`
(JengaBuilder.py:309-326): coordinates are divided by 170 and then compared against the same
threshold 170, so every pair is related (fully connected towers).
"""
from __future__ import annotations

from typing import Tuple, Union

import numpy as np
import torch

from . import engine as E
from .batch import TowerBatch
from .data import RELATION_THRESHOLD
from .network import GraphNetwork

Net = Union[GraphNetwork, "object"]   # GraphNetwork or a keras_api.KerasModel (uses its .net)


def _graph_net(net) -> GraphNetwork:
    return net if isinstance(net, GraphNetwork) else net.net


def removal_candidates(boxes_raw: np.ndarray) -> np.ndarray:
    """(n, n-1, 3): candidate i is the tower with box i removed, the others in their order
    (JengaBuilder.py:244-249)."""
    boxes_raw = np.asarray(boxes_raw, np.float64)
    n = boxes_raw.shape[0]
    if n < 2:
        raise ValueError("a removal needs at least two boxes")
    keep = ~np.eye(n, dtype=bool)
    return np.stack([boxes_raw[keep[i]] for i in range(n)])


def stability_sums(net: Net, towers_raw: np.ndarray, mode: str = "sum_prob") -> torch.Tensor:
    """(C,) Σ ŷ (or another `tower_readout` mode) of each candidate tower (C, N, 3) in raw pixels,
    one batched inference forward (`predict_stabilities` semantics, JengaBuilder.py:309-329)."""
    g = _graph_net(net)
    towers_raw = np.asarray(towers_raw, np.float64)
    objects = (towers_raw / RELATION_THRESHOLD).astype(np.float32)
    batch = TowerBatch.fully_connected(objects, device=g.device)
    with torch.no_grad():
        z = E.forward(g.flat.detach(), batch, E.RunConfig(g.mp_steps, training=False), E.Workspace(g.device))
        return E.tower_readout(z, batch, mode)


def remove_to_demolish(net: Net, boxes_raw: np.ndarray) -> Tuple[np.ndarray, int]:
    """Batched `JengaBuilder.remove_to_demolish` decision: (box_stabilities (n,), remove_index)."""
    sums = stability_sums(net, removal_candidates(boxes_raw)).cpu().numpy().astype(np.float64)
    return sums, int(np.argmin(sums))


def drop_to_demolish(net: Net, towers_with_drop_raw: np.ndarray) -> Tuple[np.ndarray, int]:
    """Batched `TowerCreator.drop_to_demolish` decision over C candidate towers (object 0 = the
    dropped box at each candidate position): (pos_stability (C,), index_min)."""
    sums = stability_sums(net, towers_with_drop_raw).cpu().numpy().astype(np.float64)
    return sums, int(np.argmin(sums))
