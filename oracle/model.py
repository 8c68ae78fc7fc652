"""CPU oracle for the propagation-network hot path — TEST INFRASTRUCTURE ONLY.

This module is a plain restatement (torch on CPU, fp64 or fp32) of the reference's
model graph, written so the HIP path can be checked against it. Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import it, and
only as the checker / the CPU baseline; the product path never routes through it.

PARITY STATUS: **parity unpinned**. The reference (Keras 2.x on TensorFlow 1.x) cannot
run in this image (``keras``/``tensorflow`` are not installed, there is no network) and it
ships no tests, no golden vectors and no trained weights. This oracle
is therefore pinned only by (a) a line-by-line restatement of the reference graph, (b)
internal consistency between three independent formulations (dense one-hot ``bmm`` exactly
as Keras builds it, an index-gather form, and a per-tower loop form), (c) known-answer
tests, and (d) committed self-generated golden vectors (``tests/golden``).

Reference anchors (``/root/reference/src``):
  * inputs & layout ............ Networks.py:22-29 (objects, sender/receiver relations, propagation)
  * endpoint gathers ........... Networks.py:32-33  senders = Rsᵀ·objects, receivers = Rrᵀ·objects
  * feature slicing ............ Networks.py:35-37, 58-71  d = r_pos − s_pos; o = (y, width)
  * MLP blocks ................. Blocks.py:20-28, 60-68  Dense(relu)…, last Dense(linear)
  * MLP sizes .................. Networks.py:46-50  rm 2→150³→150, om 2→100→100,
                                                     rmp 350→150→150→100, omp 300→100→101
  * encoder relu + dropout ..... Networks.py:75-78
  * 5 propagation steps ........ Networks.py:83-91  (shared weights each step)
  * readout .................... Networks.py:93-96  sigmoid(x[:, :, :1]) of the last step
  * loss / optimizer ........... Networks.py:101-102  Adam(lr=5e-4), binary_crossentropy
"""
from __future__ import annotations

import math
from typing import Dict, Iterable, List, Optional, Tuple

import numpy as np
import torch

# (input width, layer widths) per MLP — Networks.py:46-50 (+ Blocks.py:20-28 / 60-68)
MLP_SPECS: Dict[str, Tuple[int, List[int]]] = {
    "rm": (2, [150, 150, 150, 150]),
    "om": (2, [100, 100]),
    "rmp": (350, [150, 150, 100]),
    "omp": (300, [100, 101]),
}
STATE_DIM = 100          # Networks.py:29 / :80 ('propagation' width, "100 is the layer size")
REF_MP_STEPS = 5         # Networks.py:83
DROPOUT_RATE = 0.1       # Networks.py:77-78
RELATION_THRESHOLD = 170.0  # main.py:71 / :91


def param_shapes() -> List[Tuple[str, Tuple[int, ...]]]:
    """Ordered (name, shape) list in Keras layout: kernel (in, out), bias (out,)."""
    out = []
    for mlp, (fin, widths) in MLP_SPECS.items():
        prev = fin
        for i, w in enumerate(widths):
            out.append((f"{mlp}.{i}.kernel", (prev, w)))
            out.append((f"{mlp}.{i}.bias", (w,)))
            prev = w
    return out


def glorot_uniform_params(seed: int = 0, dtype=np.float32) -> Dict[str, np.ndarray]:
    """Keras defaults for Dense (Blocks.py:23-27): glorot_uniform kernels, zero biases.

    limit = sqrt(6 / (fan_in + fan_out)); values ~ U(-limit, limit).
    The RNG stream is numpy's, not TensorFlow's (Keras' own draws cannot be reproduced
    offline), so this matches the *distribution*, not the exact values.
    """
    rng = np.random.default_rng(seed)
    p = {}
    for name, shape in param_shapes():
        if name.endswith("kernel"):
            lim = math.sqrt(6.0 / (shape[0] + shape[1]))
            p[name] = rng.uniform(-lim, lim, size=shape).astype(dtype)
        else:
            p[name] = np.zeros(shape, dtype=dtype)
    return p


def random_params(seed: int = 0, bias_scale: float = 0.05, dtype=np.float32) -> Dict[str, np.ndarray]:
    """glorot kernels plus small random biases (so bias paths are exercised by tests)."""
    p = glorot_uniform_params(seed, dtype)
    rng = np.random.default_rng(seed + 7919)
    for name, shape in param_shapes():
        if name.endswith("bias"):
            p[name] = rng.uniform(-bias_scale, bias_scale, size=shape).astype(dtype)
    return p


def to_torch(params: Dict[str, np.ndarray], dtype=torch.float64, requires_grad=False):
    return {k: torch.tensor(np.asarray(v), dtype=dtype, requires_grad=requires_grad)
            for k, v in params.items()}


def _mlp(x: torch.Tensor, p: Dict[str, torch.Tensor], name: str) -> torch.Tensor:
    """Blocks.py:20-28 / 60-68: relu on every Dense but the last, which is linear.

    Blocks.py:43-47 reshape rows to (-1, F) — a row-wise MLP; torch broadcasting over
    the leading dims is the same computation.
    """
    n = len(MLP_SPECS[name][1])
    for i in range(n):
        x = x @ p[f"{name}.{i}.kernel"] + p[f"{name}.{i}.bias"]
        if i < n - 1:
            x = torch.relu(x)
    return x


# ---------------------------------------------------------------------------------------
# Form 1: dense one-hot bmm, literally as Networks.py builds the Keras graph.
# ---------------------------------------------------------------------------------------
def forward_dense(p, objects, Rs, Rr, prop, mp_steps: int = REF_MP_STEPS,
                  drop_r: Optional[torch.Tensor] = None, drop_o: Optional[torch.Tensor] = None,
                  return_state: bool = False):
    """Logits (B, N) of the reference model.

    objects (B,N,3)  Rs, Rr (B,N,E)  prop (B,N,100).  ``drop_r`` (B,E,150) / ``drop_o``
    (B,N,100) are multiplicative inverted-dropout masks (None = inference / dropout off).
    The reference returns sigmoid(logits)[..., None] (Networks.py:94-96).
    """
    Rs_t = Rs.transpose(1, 2)                       # Permute((2,1))  Networks.py:27-28
    Rr_t = Rr.transpose(1, 2)
    senders = torch.bmm(Rs_t, objects)              # Networks.py:32
    receivers = torch.bmm(Rr_t, objects)            # Networks.py:33
    diff = receivers[..., 0:2] - senders[..., 0:2]  # Networks.py:58-62
    obj_vec = torch.cat([objects[..., 1:2], objects[..., 2:3]], dim=-1)  # Networks.py:65-71
    c_r = torch.relu(_mlp(diff, p, "rm"))           # Networks.py:75
    c_o = torch.relu(_mlp(obj_vec, p, "om"))        # Networks.py:76
    if drop_r is not None:                          # Networks.py:77-78
        c_r = c_r * drop_r
    if drop_o is not None:
        c_o = c_o * drop_o
    P = prop
    states = [P]
    x = None
    for _ in range(mp_steps):                       # Networks.py:83
        ps = torch.bmm(Rs_t, P)                     # Networks.py:84
        pr = torch.bmm(Rr_t, P)                     # Networks.py:85
        x = _mlp(torch.cat([c_r, ps, pr], dim=-1), p, "rmp")       # Networks.py:86-87
        eff = torch.tanh(torch.bmm(Rr, x))          # Networks.py:88
        x = _mlp(torch.cat([c_o, eff, P], dim=-1), p, "omp")       # Networks.py:89-90
        P = torch.tanh(x[..., 1:] + P)              # Networks.py:91 (prop_layer = x[:,:,1:], :80)
        states.append(P)
    logits = x[..., 0]                              # Networks.py:94 sigmoid(x[:,:,:1]) -> logit
    if return_state:
        return logits, states
    return logits


# ---------------------------------------------------------------------------------------
# Form 2: compact edge list (global node indices), index gather + index_add segment sum.
# ---------------------------------------------------------------------------------------
def forward_gather(p, pos, src, dst, prop, mp_steps: int = REF_MP_STEPS,
                   drop_r: Optional[torch.Tensor] = None, drop_o: Optional[torch.Tensor] = None):
    """Same model on a flat union graph.

    pos (Nn,3) objects rows; src/dst (Ne,) int64 global node ids; prop (Nn,100).
    Returns logits (Nn,).  Mathematically identical to form 1 when every relation
    column of Rs/Rr is one-hot (inactive columns drop out: their message is never summed).
    """
    diff = pos[dst, 0:2] - pos[src, 0:2]
    obj_vec = pos[:, 1:3]
    c_r = torch.relu(_mlp(diff, p, "rm"))
    c_o = torch.relu(_mlp(obj_vec, p, "om"))
    if drop_r is not None:
        c_r = c_r * drop_r
    if drop_o is not None:
        c_o = c_o * drop_o
    P = prop
    x = None
    for _ in range(mp_steps):
        x = _mlp(torch.cat([c_r, P[src], P[dst]], dim=-1), p, "rmp")
        agg = torch.zeros(P.shape[0], x.shape[1], dtype=x.dtype).index_add_(0, dst, x)
        eff = torch.tanh(agg)
        x = _mlp(torch.cat([c_o, eff, P], dim=-1), p, "omp")
        P = torch.tanh(x[:, 1:] + P)
    return x[:, 0]


def relu_margins_gather(p, pos, src, dst, prop, tower_of_node, n_towers: int,
                        mp_steps: int = REF_MP_STEPS, drop_r=None, drop_o=None,
                        chunk_nodes: int = 1 << 15) -> np.ndarray:
    """Per tower: the smallest |pre-activation| over every ReLU its forward evaluates (fp64, dropout
    off) — rm's four (Blocks.py:20-28 + Networks.py:75), om's two (Networks.py:76), rmp's two and omp's
    one per step (Networks.py:86-90) — and the logit's distance to the BCE clip (Networks.py:102).

    A ReLU's derivative jumps at 0: an fp32 implementation whose pre-activation lands within its own
    rounding of 0 may take the other side of the kink, and then one edge's or node's term moves
    between the two sides of a gradient sum. Parity tests of the summed gradients keep towers whose
    margin is far above fp32 rounding (tests/test_gpu_chain_parity.py). Same forward as
    `forward_gather` (``drop_r`` (Ne,150) / ``drop_o`` (Nn,100): its dropout masks); evaluated over contiguous node ranges of whole towers (``chunk_nodes``) to bound
    memory. pos (Nn,3), src/dst (Ne,) global node ids, tower_of_node (Nn,) sorted tower ids."""
    tower_of_node = np.asarray(tower_of_node, np.int64)
    src = np.asarray(src, np.int64)
    dst = np.asarray(dst, np.int64)
    out = np.full(n_towers, np.inf)
    Nn = len(tower_of_node)
    e_order = np.argsort(dst, kind="stable")
    dst_sorted = dst[e_order]
    a = 0
    with torch.no_grad():
        while a < Nn:
            b = min(Nn, a + chunk_nodes)
            while b < Nn and tower_of_node[b] == tower_of_node[b - 1]:   # whole towers only
                b += 1
            e_lo, e_hi = np.searchsorted(dst_sorted, [a, b])
            ei = np.sort(e_order[e_lo:e_hi])
            s_ = torch.as_tensor(src[ei] - a)
            d_ = torch.as_tensor(dst[ei] - a)
            et = torch.as_tensor(tower_of_node[dst[ei]])
            nt = torch.as_tensor(tower_of_node[a:b])
            x = torch.as_tensor(np.asarray(pos[a:b], np.float64))
            P = torch.as_tensor(np.asarray(prop[a:b], np.float64))
            marg = torch.full((n_towers,), float("inf"), dtype=torch.float64)

            def note(pre, rows_tower):
                m = pre.abs().amin(dim=1)
                marg.scatter_reduce_(0, rows_tower, m, reduce="amin")

            h = x[d_, 0:2] - x[s_, 0:2]
            for i in range(4):
                h = h @ p[f"rm.{i}.kernel"] + p[f"rm.{i}.bias"]
                note(h, et)
                h = torch.relu(h)
            c_r = h if drop_r is None else h * torch.as_tensor(np.asarray(drop_r[ei], np.float64))
            h = x[:, 1:3]
            for i in range(2):
                h = h @ p[f"om.{i}.kernel"] + p[f"om.{i}.bias"]
                note(h, nt)
                h = torch.relu(h)
            c_o = h if drop_o is None else h * torch.as_tensor(np.asarray(drop_o[a:b], np.float64))
            z = None
            for _ in range(mp_steps):
                h = torch.cat([c_r, P[s_], P[d_]], dim=-1)
                for i in range(2):
                    h = h @ p[f"rmp.{i}.kernel"] + p[f"rmp.{i}.bias"]
                    note(h, et)
                    h = torch.relu(h)
                msg = h @ p["rmp.2.kernel"] + p["rmp.2.bias"]
                agg = torch.zeros(b - a, msg.shape[1], dtype=msg.dtype).index_add_(0, d_, msg)
                h = torch.cat([c_o, torch.tanh(agg), P], dim=-1) @ p["omp.0.kernel"] + p["omp.0.bias"]
                note(h, nt)
                xo = torch.relu(h) @ p["omp.1.kernel"] + p["omp.1.bias"]
                P = torch.tanh(xo[:, 1:] + P)
                z = xo[:, 0]
            note((z.abs() - LOGIT_CLIP)[:, None], nt)
            out = np.minimum(out, marg.numpy())
            a = b
    return out


# ---------------------------------------------------------------------------------------
# Form 3: plain per-tower python loop with explicit sums (small cases only).
# ---------------------------------------------------------------------------------------
def forward_loop_numpy(params: Dict[str, np.ndarray], objects: np.ndarray, Rs: np.ndarray,
                       Rr: np.ndarray, prop: np.ndarray, mp_steps: int = REF_MP_STEPS) -> np.ndarray:
    """fp64 numpy, one tower and one relation at a time (no batched matmul over relations)."""
    P64 = {k: np.asarray(v, np.float64) for k, v in params.items()}

    def mlp(x, name):
        n = len(MLP_SPECS[name][1])
        for i in range(n):
            x = x @ P64[f"{name}.{i}.kernel"] + P64[f"{name}.{i}.bias"]
            if i < n - 1:
                x = np.maximum(x, 0.0)
        return x

    B, N, _ = objects.shape
    E = Rs.shape[2]
    out = np.zeros((B, N))
    for b in range(B):
        obj = objects[b].astype(np.float64)
        c_o = np.maximum(mlp(obj[:, 1:3], "om"), 0.0)
        rel = []
        for k in range(E):
            s_vec = sum(Rs[b, i, k] * obj[i] for i in range(N))
            r_vec = sum(Rr[b, i, k] * obj[i] for i in range(N))
            rel.append(np.maximum(mlp((r_vec[0:2] - s_vec[0:2])[None], "rm")[0], 0.0))
        P = prop[b].astype(np.float64)
        x = None
        for _ in range(mp_steps):
            eff = np.zeros((N, STATE_DIM))
            msgs = []
            for k in range(E):
                ps = sum(Rs[b, i, k] * P[i] for i in range(N))
                pr = sum(Rr[b, i, k] * P[i] for i in range(N))
                msgs.append(mlp(np.concatenate([rel[k], ps, pr])[None], "rmp")[0])
            for i in range(N):
                acc = np.zeros(STATE_DIM)
                for k in range(E):
                    acc = acc + Rr[b, i, k] * msgs[k]
                eff[i] = np.tanh(acc)
            x = mlp(np.concatenate([c_o, eff, P], axis=1), "omp")
            P = np.tanh(x[:, 1:] + P)
        out[b] = x[:, 0]
    return out


# ---------------------------------------------------------------------------------------
# Keras semantics: loss, metric, optimizer (Networks.py:101-102).
# ---------------------------------------------------------------------------------------
KERAS_EPS = 1e-7
LOGIT_CLIP = math.log((1.0 - KERAS_EPS) / KERAS_EPS)   # ≈ 16.118


def keras_bce_from_logits(logits: torch.Tensor, target: torch.Tensor) -> torch.Tensor:
    """Keras 2.x ``binary_crossentropy`` on the model's sigmoid output, mean over B·N.

    keras.backend.binary_crossentropy clips ŷ to [eps, 1-eps], converts back to a logit
    and calls sigmoid_cross_entropy_with_logits; in exact arithmetic that is BCE-with-logits
    on clamp(z, ±ln((1-eps)/eps)), with zero gradient where the clamp is active.
    """
    z = torch.clamp(logits, -LOGIT_CLIP, LOGIT_CLIP)
    per = torch.clamp(z, min=0) - z * target + torch.log1p(torch.exp(-torch.abs(z)))
    return per.mean()


def keras_bce_grad(logits: np.ndarray, target: np.ndarray) -> Tuple[float, np.ndarray]:
    """(loss, dloss/dlogit) in fp64 numpy; mean over all elements."""
    z64 = np.asarray(logits, np.float64)
    t = np.asarray(target, np.float64)
    z = np.clip(z64, -LOGIT_CLIP, LOGIT_CLIP)
    per = np.maximum(z, 0) - z * t + np.log1p(np.exp(-np.abs(z)))
    n = z.size
    g = (1.0 / (1.0 + np.exp(-z64)) - t) / n
    g = np.where(np.abs(z64) < LOGIT_CLIP, g, 0.0)
    return float(per.mean()), g


def binary_accuracy(probs: np.ndarray, target: np.ndarray) -> float:
    """Keras ``binary_accuracy``: mean(round(ŷ) == y)."""
    return float(np.mean((np.asarray(probs) > 0.5).astype(np.float64) == np.asarray(target)))


class KerasAdam:
    """Keras 2.x Adam (lr=5e-4, β1=0.9, β2=0.999, epsilon=K.epsilon()=1e-7, decay=0).

    t = iterations + 1; lr_t = lr·sqrt(1-β2^t)/(1-β1^t);
    m = β1 m + (1-β1) g;  v = β2 v + (1-β2) g²;  p -= lr_t · m / (sqrt(v) + eps)
    """

    def __init__(self, lr=5e-4, beta1=0.9, beta2=0.999, eps=KERAS_EPS, l2: float = 0.0):
        self.lr, self.b1, self.b2, self.eps, self.l2 = lr, beta1, beta2, eps, l2
        self.t = 0
        self.m = None
        self.v = None

    def step(self, params: np.ndarray, grads: np.ndarray) -> np.ndarray:
        params = np.asarray(params, np.float64)
        g = np.asarray(grads, np.float64) + 2.0 * self.l2 * params
        if self.m is None:
            self.m = np.zeros_like(params)
            self.v = np.zeros_like(params)
        self.t += 1
        lr_t = self.lr * math.sqrt(1.0 - self.b2 ** self.t) / (1.0 - self.b1 ** self.t)
        self.m = self.b1 * self.m + (1.0 - self.b1) * g
        self.v = self.b2 * self.v + (1.0 - self.b2) * g * g
        return params - lr_t * self.m / (np.sqrt(self.v) + self.eps)


# ---------------------------------------------------------------------------------------
# Convenience: gradients of the mean BCE w.r.t. every parameter (autograd on the oracle).
# ---------------------------------------------------------------------------------------
def loss_and_grads(params: Dict[str, np.ndarray], objects, Rs, Rr, prop, target,
                   mp_steps: int = REF_MP_STEPS, dtype=torch.float64, form: str = "dense",
                   src=None, dst=None, drop_r=None, drop_o=None):
    """Returns (loss, logits (np), grads dict (np)) using torch autograd on the oracle."""
    tp = to_torch(params, dtype=dtype, requires_grad=True)
    if form == "dense":
        logits = forward_dense(tp, torch.as_tensor(objects, dtype=dtype), torch.as_tensor(Rs, dtype=dtype),
                               torch.as_tensor(Rr, dtype=dtype), torch.as_tensor(prop, dtype=dtype),
                               mp_steps, drop_r=None if drop_r is None else torch.as_tensor(drop_r, dtype=dtype),
                               drop_o=None if drop_o is None else torch.as_tensor(drop_o, dtype=dtype))
    else:
        logits = forward_gather(tp, torch.as_tensor(objects, dtype=dtype), torch.as_tensor(src),
                                torch.as_tensor(dst), torch.as_tensor(prop, dtype=dtype), mp_steps,
                                drop_r=None if drop_r is None else torch.as_tensor(drop_r, dtype=dtype),
                                drop_o=None if drop_o is None else torch.as_tensor(drop_o, dtype=dtype))
    loss = keras_bce_from_logits(logits, torch.as_tensor(target, dtype=dtype).reshape(logits.shape))
    loss.backward()
    grads = {k: v.grad.detach().numpy().copy() for k, v in tp.items()}
    return float(loss.detach()), logits.detach().numpy(), grads


# ---------------------------------------------------------------------------------------
# Relation matrices exactly as the training driver builds them (main.py:66-81).
# ---------------------------------------------------------------------------------------
def relation_matrices(pos_raw: np.ndarray, threshold: Optional[float] = RELATION_THRESHOLD):
    """Dense (B,N,E) sender/receiver one-hot matrices.

    pos_raw (B,N,>=2) in the units the threshold applies to; edge k enumerates ordered pairs
    (m, j), m != j, sender-major (main.py:72-81). threshold=None → fully connected.
    """
    B, N = pos_raw.shape[:2]
    E = N * (N - 1)
    Rs = np.zeros((B, N, E))
    Rr = np.zeros((B, N, E))
    cnt = 0
    for m in range(N):
        for j in range(N):
            if m != j:
                if threshold is None:
                    inzz = np.ones(B, dtype=bool)
                else:
                    inzz = np.linalg.norm(pos_raw[:, m, 0:2] - pos_raw[:, j, 0:2], axis=1) < threshold
                Rr[inzz, j, cnt] = 1.0
                Rs[inzz, m, cnt] = 1.0
                cnt += 1
    return Rs, Rr


def dense_to_edges(Rs: np.ndarray, Rr: np.ndarray):
    """Active (tower, slot, sender, receiver) for one-hot relation columns (test helper)."""
    out = []
    B, N, E = Rs.shape
    for b in range(B):
        for k in range(E):
            s = np.nonzero(Rs[b, :, k])[0]
            r = np.nonzero(Rr[b, :, k])[0]
            if len(r):
                out.append((b, k, int(s[0]), int(r[0])))
    return out
