"""Input builders: synthetic Jenga towers, relation matrices, stability labels, JSON trajectories.

Mirrors the reference's data producers and driver preprocessing (no physics):
  * tower geometry ........ src/JengaBuilder.py:50-61 (constants), :137-192 (create_world),
                            :223-233 (remove_object) — positions of the first recorded frame
  * relation matrices ..... src/main.py:66-81 (raw-pixel distance < 170, sender-major slots) and
                            src/JengaBuilder.py:309-326 (normalised coords vs 170 → fully connected)
  * stability labels ...... src/main.py:8-23 (Σ‖Δpos‖ over frames < 0.5 px ⇒ stable)
  * trajectories on disk .. src/JengaBuilder.py:128-135, :366-371 (JSON [traj][obj][frame][x,y,w]),
                            src/main.py:39-63 (load, drop empty, pad frames with the last frame)
  * normalisation ......... src/main.py:91 (boxes / 170)
"""
from __future__ import annotations

import json
import random
from typing import List, Optional, Tuple

import numpy as np

RELATION_THRESHOLD = 170.0        # main.py:71
# JengaBuilder.py:50-61
BOTTOM_EDGE = 70
LEFT_MOST = 400
RIGHT_MOST = 1500 - 400
RECT_HEIGHT = 80
RECT_WIDTH_MIN = 50
RECT_WIDTH_RANGE = 250
RECT_WIDTH_AVERAGE = (RECT_WIDTH_MIN + RECT_WIDTH_RANGE) / 2
MAX_SPACE_RECTS = 50


def jenga_tower(n: int, rng: random.Random) -> np.ndarray:
    """One tower of n boxes [x, y, w] in pixels, laid out like JengaBuilder.create_world."""
    boxes: List[List[Tuple[float, float, float]]] = []
    layer = -1
    while n > 0:
        layer += 1
        boxes.append([])
        if layer == 0:
            right_edge, left_edge = RIGHT_MOST, LEFT_MOST
        else:
            xs = [b[0] for b in boxes[layer - 1]]
            right_edge, left_edge = max(xs), min(xs)
        y = BOTTOM_EDGE + RECT_HEIGHT / 2 + RECT_HEIGHT * layer
        if right_edge == left_edge:  # previous layer holds one box (JengaBuilder.py:159-167)
            x = rng.randint(int(left_edge - RECT_WIDTH_MIN / 2), int(left_edge + RECT_WIDTH_MIN / 2))
            w = rng.randint(RECT_WIDTH_MIN, RECT_WIDTH_MIN + RECT_WIDTH_RANGE)
            boxes[layer].append((float(x), BOTTOM_EDGE + int(RECT_HEIGHT / 2) + RECT_HEIGHT * layer, float(w)))
            n -= 1
            continue
        left_edge -= (layer > 0) * int(RECT_WIDTH_AVERAGE / 2)   # JengaBuilder.py:171
        w = rng.randint(RECT_WIDTH_MIN, RECT_WIDTH_MIN + RECT_WIDTH_RANGE)
        left_edge += w
        while left_edge - w / 2 < right_edge and n > 0:          # JengaBuilder.py:174-184
            boxes[layer].append((left_edge - w / 2, y, float(w)))
            n -= 1
            left_edge += rng.randint(0, MAX_SPACE_RECTS)
            w = rng.randint(RECT_WIDTH_MIN, RECT_WIDTH_MIN + RECT_WIDTH_RANGE)
            left_edge += w
        if not boxes[layer]:   # a first box wider than the narrow layer below: centre one box on it
            boxes[layer].append(((left_edge - w + right_edge) / 2, y, float(w)))
            n -= 1
    return np.array([b for layer_boxes in boxes for b in layer_boxes], dtype=np.float64)


def synthetic_towers(n_towers: int, n_objects: int, seed: int = 0, remove_one: bool = True) -> np.ndarray:
    """(B, N, 3) raw-pixel [x, y, w]: build N+1 boxes and remove one at random (the Jenga
    trajectory records the tower after remove_object, JengaBuilder.py:223-233)."""
    rng = random.Random(seed)
    out = np.zeros((n_towers, n_objects, 3))
    for b in range(n_towers):
        t = jenga_tower(n_objects + (1 if remove_one else 0), rng)
        if remove_one:
            t = np.delete(t, rng.randint(0, len(t) - 1), axis=0)
        out[b] = t
    return out


def _draw(u: np.ndarray, lo: int, hi: int) -> np.ndarray:
    """randint(lo, hi) inclusive from uniforms in [0, 1)."""
    return lo + np.minimum(np.floor(u * (hi - lo + 1)), hi - lo).astype(np.int64)


def draws_per_tower(n_objects: int) -> int:
    """Upper bound on the random draws one tower of `n_objects` (+1 removed) consumes below: per box
    a width and a gap, per layer one width, plus one x offset and the removal index."""
    return 4 * (n_objects + 1) + 4


def jenga_towers_from_draws(u: np.ndarray, n_objects: int, remove_one: bool = True) -> np.ndarray:
    """Vectorised `jenga_tower` over T towers at once: (T, n_objects, 3) raw-pixel [x, y, w].

    Each tower t consumes its own row u[t] of uniforms in [0, 1) strictly in order (counter c[t]),
    in the same sequence the scalar builder draws (JengaBuilder.py:159-184: layer width, then per
    box the gap and the next width; a one-box layer below draws the x offset, then the width), so
    the scalar `jenga_tower` fed one row gives the same tower. All towers advance in lockstep: each
    iteration either opens a layer or places/ends one box of the open layer."""
    T = u.shape[0]
    n_build = n_objects + (1 if remove_one else 0)
    ar = np.arange(T)
    c = np.zeros(T, np.int64)

    def take(lo, hi, m):
        v = _draw(u[ar[m], c[m]], lo, hi)
        c[m] += 1
        return v

    out = np.zeros((T, n_build, 3))
    placed = np.zeros(T, np.int64)
    layer = np.full(T, -1, np.int64)
    in_layer = np.zeros(T, bool)               # a multi-box layer is open
    cnt = np.zeros(T, np.int64)                # boxes in the open layer
    prev_min = np.zeros(T)
    prev_max = np.zeros(T)
    cur_min = np.full(T, np.inf)
    cur_max = np.full(T, -np.inf)
    left = np.zeros(T)
    right = np.zeros(T)
    w = np.zeros(T)
    y = np.zeros(T)

    def place(m, x, yy, ww):
        i = np.nonzero(m)[0]
        out[i, placed[i], 0] = x
        out[i, placed[i], 1] = yy
        out[i, placed[i], 2] = ww
        placed[i] += 1
        cur_min[i] = np.minimum(cur_min[i], x)
        cur_max[i] = np.maximum(cur_max[i], x)

    while True:
        todo = placed < n_build
        if not todo.any():
            break
        # ---- open a layer
        op = todo & ~in_layer
        if op.any():
            layer[op] += 1
            first = op & (layer == 0)
            later = op & (layer > 0)
            prev_min[later], prev_max[later] = cur_min[later], cur_max[later]
            right[first], left[first] = RIGHT_MOST, LEFT_MOST
            right[later], left[later] = prev_max[later], prev_min[later]
            cur_min[op], cur_max[op] = np.inf, -np.inf
            y[op] = BOTTOM_EDGE + RECT_HEIGHT / 2 + RECT_HEIGHT * layer[op]
            single = op & (right == left)
            if single.any():                   # JengaBuilder.py:159-167
                xs = left[single]
                x = (np.floor(xs - RECT_WIDTH_MIN / 2) + take(0, RECT_WIDTH_MIN, single)).astype(np.float64)
                ww = take(RECT_WIDTH_MIN, RECT_WIDTH_MIN + RECT_WIDTH_RANGE, single).astype(np.float64)
                place(single, x, BOTTOM_EDGE + int(RECT_HEIGHT / 2) + RECT_HEIGHT * layer[single], ww)
                # the layer is complete (stays closed): next iteration opens the next one
            multi = op & ~single
            if multi.any():                    # JengaBuilder.py:171-173
                left[multi] -= (layer[multi] > 0) * int(RECT_WIDTH_AVERAGE / 2)
                w[multi] = take(RECT_WIDTH_MIN, RECT_WIDTH_MIN + RECT_WIDTH_RANGE, multi)
                left[multi] += w[multi]
                in_layer[multi] = True
                cnt[multi] = 0
            continue
        # ---- one step of the open layers: place a box or close the layer (JengaBuilder.py:174-184)
        go = todo & in_layer & (left - w / 2 < right)
        if go.any():
            place(go, left[go] - w[go] / 2, y[go], w[go].copy())
            cnt[go] += 1
            # the scalar loop draws the gap and the next width even after its last box
            left[go] += take(0, MAX_SPACE_RECTS, go)
            w[go] = take(RECT_WIDTH_MIN, RECT_WIDTH_MIN + RECT_WIDTH_RANGE, go)
            left[go] += w[go]
            in_layer[go & (placed >= n_build)] = False
        stop = todo & in_layer & ~go
        if stop.any():
            empty = stop & (cnt == 0)
            if empty.any():                    # first box wider than the narrow layer below
                place(empty, (left[empty] - w[empty] + right[empty]) / 2, y[empty], w[empty].copy())
            in_layer[stop] = False
    if not remove_one:
        return out
    r = take(0, n_build - 1, np.ones(T, bool))
    keep = np.ones((T, n_build), bool)
    keep[ar, r] = False
    return out[keep].reshape(T, n_objects, 3)


def synthetic_towers_fast(n_towers: int, n_objects: int, seed: int = 0, remove_one: bool = True) -> np.ndarray:
    """`synthetic_towers`' geometry for large batches: (B, N, 3) raw-pixel towers from a numpy
    uniform table, built by the vectorised lockstep builder (≈ 100× faster than the per-tower loop;
    a different random stream, the same distribution)."""
    u = np.random.default_rng(seed).random((n_towers, draws_per_tower(n_objects)))
    return jenga_towers_from_draws(u, n_objects, remove_one)


def relation_matrices(boxes_raw: np.ndarray, threshold: Optional[float] = RELATION_THRESHOLD):
    """Dense sender/receiver one-hot matrices (B, N, E), E = N(N-1), exactly as main.py:66-81
    (threshold on raw-pixel frame-0 distance) — vectorised over towers and slots.
    threshold=None → fully connected (the inference path of JengaBuilder.py:309-326)."""
    B, N = boxes_raw.shape[:2]
    m_idx, j_idx = np.nonzero(~np.eye(N, dtype=bool))          # sender-major slot order
    E = len(m_idx)
    if threshold is None:
        active = np.ones((B, E), dtype=bool)
    else:
        d = np.linalg.norm(boxes_raw[:, m_idx, 0:2] - boxes_raw[:, j_idx, 0:2], axis=2)
        active = d < threshold
    Rs = np.zeros((B, N, E), dtype=np.float32)
    Rr = np.zeros((B, N, E), dtype=np.float32)
    bb, kk = np.nonzero(active)
    Rs[bb, m_idx[kk], kk] = 1.0
    Rr[bb, j_idx[kk], kk] = 1.0
    return Rs, Rr


def calculate_stability(boxes: np.ndarray, threshold: float = 0.5) -> np.ndarray:
    """main.py:8-23: boxes (T, F, N, >=2) → y (T, N, 1); stable iff Σ_f ‖pos_f − pos_{f+1}‖ < 0.5."""
    step = np.linalg.norm(boxes[:, 1:, :, 0:2] - boxes[:, :-1, :, 0:2], axis=3)   # (T, F-1, N)
    return (step.sum(axis=1) < threshold).astype(np.float64)[..., None]


def load_trajectories(path: str, n_objects: int, object_dim: int = 3) -> np.ndarray:
    """main.py:39-63: JSON [traj][obj][frame][x,y,(w)] → (T, F, N, object_dim); F = max over
    trajectories of object 0's frame count (main.py:46-47); each object is truncated to F or
    padded with its last frame; empty trajectories dropped (main.py:44)."""
    with open(path) as f:
        data = json.load(f)
    data = [d for d in data if len(d) != 0]
    n_frame = max(len(t[0]) for t in data)
    boxes = np.zeros((len(data), n_frame, n_objects, object_dim))
    for t, traj in enumerate(data):
        for o in range(n_objects):
            fr = np.asarray(traj[o], dtype=np.float64)[:n_frame, :object_dim]   # main.py:55-63 truncates/pads
            boxes[t, :len(fr), o] = fr
            boxes[t, len(fr):, o] = fr[-1]
    return boxes


def training_arrays(boxes: np.ndarray, threshold: float = RELATION_THRESHOLD):
    """The dicts main.py:92-93 passes to fit: relations from raw frame 0, then /170."""
    Rs, Rr = relation_matrices(boxes[:, 0], threshold)
    y = calculate_stability(boxes)
    objects = (boxes[:, 0] / RELATION_THRESHOLD).astype(np.float32)
    prop = np.zeros(objects.shape[:2] + (100,), np.float32)
    return ({"objects": objects, "sender_relations": Rs, "receiver_relations": Rr, "propagation": prop},
            {"target": y.astype(np.float32)})


def synthetic_batch(n_towers: int, n_objects: int, seed: int = 0, fully_connected: bool = True):
    """Synthetic (objects /170, Rs, Rr, prop, target) for benchmarks: Jenga geometry, Bernoulli labels."""
    raw = synthetic_towers(n_towers, n_objects, seed)
    Rs, Rr = relation_matrices(raw, None if fully_connected else RELATION_THRESHOLD)
    rng = np.random.default_rng(seed + 1)
    target = rng.integers(0, 2, size=(n_towers, n_objects)).astype(np.float32)
    objects = (raw / RELATION_THRESHOLD).astype(np.float32)
    prop = np.zeros((n_towers, n_objects, 100), np.float32)
    return objects, Rs, Rr, prop, target


def ragged_batch(n_towers: int, n_min: int, n_max: int, seed: int = 0,
                 threshold: Optional[float] = RELATION_THRESHOLD):
    """BASELINE config 4's input: towers of U{n_min..n_max} Jenga boxes in random order, relations
    from the raw positions (distance < threshold, main.py:71-81; None = fully connected), objects /170.

    Returns the compact edge form `TowerBatch.from_edges` takes: (pos (Nn, 3) f32, tower_nodes (T,),
    src (Ne,), dst (Ne,), tower_edges (T,), raw (list of (N_t, 3) pixel arrays)). Edges are tower-major
    and sender-major inside a tower (the slot order of main.py:72-81). Vectorised per tower size
    (geometry from `synthetic_towers_fast`: 2^20 towers build in seconds)."""
    rng = np.random.default_rng(seed)
    sizes = rng.integers(n_min, n_max + 1, size=n_towers).astype(np.int32)
    off = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
    pos = np.zeros((int(off[-1]), 3), np.float32)
    raw_list = [None] * n_towers
    e_tower, e_src, e_dst = [], [], []
    for n in range(n_min, n_max + 1):
        idx = np.nonzero(sizes == n)[0]
        if len(idx) == 0:
            continue
        raw = synthetic_towers_fast(len(idx), n, seed=seed * 1000 + n)
        rows = off[idx][:, None] + np.arange(n)[None, :]
        pos[rows.reshape(-1)] = (raw / RELATION_THRESHOLD).reshape(-1, 3)
        for j, t in enumerate(idx):
            raw_list[t] = raw[j]
        m_idx, j_idx = np.nonzero(~np.eye(n, dtype=bool))
        if threshold is None:
            keep = np.ones((len(idx), len(m_idx)), bool)
        else:
            keep = np.linalg.norm(raw[:, m_idx, 0:2] - raw[:, j_idx, 0:2], axis=2) < threshold
        tt, kk = np.nonzero(keep)
        e_tower.append(idx[tt])
        e_src.append(off[idx[tt]] + m_idx[kk])
        e_dst.append(off[idx[tt]] + j_idx[kk])
    et = np.concatenate(e_tower) if e_tower else np.zeros(0, np.int64)
    order = np.argsort(et, kind="stable")      # tower-major, slot order kept inside a tower
    src = np.concatenate(e_src)[order].astype(np.int32) if e_src else np.zeros(0, np.int32)
    dst = np.concatenate(e_dst)[order].astype(np.int32) if e_dst else np.zeros(0, np.int32)
    tower_edges = np.bincount(et, minlength=n_towers).astype(np.int32)
    return pos, sizes, src, dst, tower_edges, raw_list


def edge_slice(pos, tower_nodes, src, dst, tower_edges, a: int, b: int):
    """Towers [a, b) of a compact edge-form batch (as `ragged_batch` returns), node ids rebased to 0:
    a micro-batch or a rank's shard of it."""
    off = np.concatenate([[0], np.cumsum(tower_nodes)]).astype(np.int64)
    eoff = np.concatenate([[0], np.cumsum(tower_edges)]).astype(np.int64)
    n0, n1, e0, e1 = off[a], off[b], eoff[a], eoff[b]
    return (pos[n0:n1], tower_nodes[a:b], (src[e0:e1] - n0).astype(np.int32), (dst[e0:e1] - n0).astype(np.int32),
            tower_edges[a:b])
