"""bf16-operand emulation of the engine's SPWGNN_MATH_BF16 arithmetic — TEST INFRASTRUCTURE ONLY.

SPWGNN_MATH_BF16 (include/spwgnn.h, "BF16") is BASELINE.json configs 3–4's arithmetic: every matrix
product's two operands are rounded to bf16 (round-to-nearest-even) and the products are accumulated
in fp32; everything that is not a matrix product (bias adds, relu/tanh, the step-invariant sums,
Adam) stays fp32. This module restates that definition on the reference graph
(Networks.py:32-96, Blocks.py:20-28/60-68) in the factored algebra the engine computes (DESIGN.md §2,
each step an identity in real arithmetic):

  * rmp layer 1 split:  [c_r | P_s | P_r]·W1 + b1 = (c_r·W1a + b1) + (P·W1b)[s] + (P·W1c)[r]
  * rmp layer 3 behind the receiver sum:  Σ_{k→i}(h2_k·W3 + b3) = [Σ h2_k | deg_i]·[W3; b3]
  * c_o·Wo1c (omp.0's object-encoding block, Networks.py:89) formed once and reused every step,

so the rounding points are those of the matrix products the engine runs (which operand a product
sees is a property of the factored form, not of the kernels' tiling):

  forward  rm.1-3, W1a, om.1, W1b/W1c, W2, [W3; b3], Wo1c/Wo1a/Wo1p, Wo2 on bf16 operands;
           rm.0 / om.0 (2-wide inputs) in fp32; the receiver sum adds bf16(h2_k) in fp32 (a one-hot
           product); the stored step-invariant A and the per-step U = P·W1b, V = P·W1c are bf16
           (training: rounded once when stored, then summed in fp32 into h1)
  backward every activation-gradient product on bf16(dY) and bf16(Wᵀ); every weight gradient
           bf16(X)ᵀ·bf16(dY), bias gradients Σ bf16(dY) (the ones column of X); the sender/receiver
           sums of dh1pre (into dU/dV) add bf16 values; dA = Σ_s dh1pre_s in fp32

Accumulation here is fp64 (the products of bf16 values are exact in both), so the emulator differs
from the engine only by fp32 accumulation order and by the rare operand that sits within fp32
rounding of a bf16 rounding boundary — far below the bf16 rounding itself.
"""
from __future__ import annotations

from typing import Dict, Optional

import numpy as np
import torch

from . import model as O


ROUND = True   # False: the same factored graph without rounding (checked against model.forward_gather)
KBLOCK = 0     # > 0: every product accumulated as a running sum of k-blocks of this size (an fp32
               # accumulator walking the contraction in MFMA-like blocks); 0: one library matmul


def mm(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """a @ b, accumulated in KBLOCK-sized k-blocks in order when KBLOCK > 0."""
    k = a.shape[1]
    if KBLOCK <= 0 or k <= KBLOCK:
        return a @ b
    acc = a[:, 0:KBLOCK] @ b[0:KBLOCK]
    for s in range(KBLOCK, k, KBLOCK):
        acc = acc + a[:, s:s + KBLOCK] @ b[s:s + KBLOCK]
    return acc


def b16(x: torch.Tensor) -> torch.Tensor:
    """Round to bf16 (RNE) and back, in x's dtype."""
    if not ROUND:
        return x
    return x.to(torch.float32).to(torch.bfloat16).to(x.dtype)


class _MM(torch.autograd.Function):
    """Y = bf16(X)·bf16(W); dX = bf16(dY)·bf16(W)ᵀ; dW = bf16(X)ᵀ·bf16(dY)."""

    @staticmethod
    def forward(ctx, x, w):
        xb, wb = b16(x), b16(w)
        ctx.save_for_backward(xb, wb)
        return mm(xb, wb)

    @staticmethod
    def backward(ctx, g):
        xb, wb = ctx.saved_tensors
        gb = b16(g)
        return mm(gb, wb.T), mm(xb.T, gb)


class _Bias(torch.autograd.Function):
    """Y = X + b (fp32); db = Σ_rows bf16(dY) (the weight-gradient kernels' ones column)."""

    @staticmethod
    def forward(ctx, x, b):
        return x + b

    @staticmethod
    def backward(ctx, g):
        return g, b16(g).reshape(-1, g.shape[-1]).sum(0)


class _Dense32(torch.autograd.Function):
    """rm.0 / om.0 on 2-wide inputs: fp32 forward; gradients as a weight-gradient kernel computes them,
    dW = bf16([x])ᵀ·bf16(dY), db = Σ bf16(dY). dx is not needed (x is an input)."""

    @staticmethod
    def forward(ctx, x, w, b):
        ctx.save_for_backward(x)
        return x @ w + b

    @staticmethod
    def backward(ctx, g):
        (x,) = ctx.saved_tensors
        gb = b16(g)
        return None, b16(x).T @ gb, gb.sum(0)


class _Round(torch.autograd.Function):
    """bf16(x) with an identity backward: a stored bf16 copy (A) or a one-hot product's operand
    (h2 in the receiver sum), whose gradient the engine passes on unrounded."""

    @staticmethod
    def forward(ctx, x):
        return b16(x)

    @staticmethod
    def backward(ctx, g):
        return g


class _Gather(torch.autograd.Function):
    """U[idx] with the scatter of the backward on bf16(dY) (the one-hot sender/receiver sums)."""

    @staticmethod
    def forward(ctx, u, idx):
        ctx.save_for_backward(idx)
        ctx.n = u.shape[0]
        return u[idx]

    @staticmethod
    def backward(ctx, g):
        (idx,) = ctx.saved_tensors
        out = torch.zeros(ctx.n, g.shape[1], dtype=g.dtype).index_add_(0, idx, b16(g))
        return out, None


def dense(x, p, name, relu):
    y = _Bias.apply(_MM.apply(x, p[name + ".kernel"]), p[name + ".bias"])
    return torch.relu(y) if relu else y


def forward(p: Dict[str, torch.Tensor], pos, src, dst, prop, mp_steps: int = O.REF_MP_STEPS,
            drop_r: Optional[torch.Tensor] = None, drop_o: Optional[torch.Tensor] = None,
            training: bool = True) -> torch.Tensor:
    """Logits (Nn,) of the bf16-operand engine arithmetic. pos (Nn, 3) objects rows, src/dst (Ne,)
    int64 global node ids, prop (Nn, 100); drop_r (Ne, 150) / drop_o (Nn, 100) multiplicative masks.
    `training` = the A, U and V arrays are stored (and read) as bf16, as the engine's bf16 training
    forward does."""
    Nn = pos.shape[0]
    # encoders (Networks.py:58-78)
    d = pos[dst, 0:2] - pos[src, 0:2]
    z1 = torch.relu(_Dense32.apply(d, p["rm.0.kernel"], p["rm.0.bias"]))
    z2 = dense(z1, p, "rm.1", True)
    z3 = dense(z2, p, "rm.2", True)
    c_r = dense(z3, p, "rm.3", True)               # rm's last Dense is linear; relu from Networks.py:75
    zo1 = torch.relu(_Dense32.apply(pos[:, 1:3], p["om.0.kernel"], p["om.0.bias"]))
    c_o = dense(zo1, p, "om.1", True)
    if drop_r is not None:
        c_r = c_r * drop_r
    if drop_o is not None:
        c_o = c_o * drop_o
    W1 = p["rmp.0.kernel"]
    A = _Bias.apply(_MM.apply(c_r, W1[0:150]), p["rmp.0.bias"])
    if training:
        A = _Round.apply(A)
    Wo1 = p["omp.0.kernel"]
    # c_o·Wo1c + bo1, once: its gradient is Σ_s do1_s, rounded once by the products
    cw = _Bias.apply(_MM.apply(c_o, Wo1[0:100]), p["omp.0.bias"])
    W3b = torch.cat([p["rmp.2.kernel"], p["rmp.2.bias"][None, :]], 0)        # [W3; b3]: 151 × 100
    deg = torch.zeros(Nn, 1, dtype=pos.dtype).index_add_(0, dst, torch.ones(len(dst), 1, dtype=pos.dtype))
    P = prop
    x = None
    for _ in range(mp_steps):                       # Networks.py:83-91
        U = _MM.apply(P, W1[150:250])
        V = _MM.apply(P, W1[250:350])
        if training:                                # stored rounded, like A
            U, V = _Round.apply(U), _Round.apply(V)
        h1 = torch.relu(A + _Gather.apply(U, src) + _Gather.apply(V, dst))
        h2 = dense(h1, p, "rmp.1", True)
        H2s = torch.zeros(Nn, 150, dtype=pos.dtype).index_add(0, dst, _Round.apply(h2))
        a = torch.tanh(_MM.apply(torch.cat([H2s, deg], 1), W3b))             # Networks.py:88
        o1 = torch.relu(cw + _MM.apply(a, Wo1[100:200]) + _MM.apply(P, Wo1[200:300]))
        x = dense(o1, p, "omp.1", False)
        P = torch.tanh(x[:, 1:] + P)                # Networks.py:91
    return x[:, 0]


def loss_and_grads(params: Dict[str, np.ndarray], pos, src, dst, prop, target, mp_steps: int = O.REF_MP_STEPS,
                   drop_r=None, drop_o=None, training: bool = True, dtype=torch.float64, kblock: int = 0):
    """(loss, logits, grads) of the Keras BCE (Networks.py:102) on the bf16-operand emulation.

    `dtype` is the accumulation type (float64: the emulator proper; float32 with `kblock` > 0: another
    valid implementation of the same bf16 definition, summing each product in k-blocks of that size)."""
    global KBLOCK
    tp = O.to_torch(params, dtype=dtype, requires_grad=True)
    t = lambda a: None if a is None else torch.as_tensor(np.ascontiguousarray(a), dtype=dtype)
    old, KBLOCK = KBLOCK, kblock
    try:
        z = forward(tp, t(pos), torch.as_tensor(np.asarray(src), dtype=torch.long),
                    torch.as_tensor(np.asarray(dst), dtype=torch.long), t(prop), mp_steps, t(drop_r), t(drop_o),
                    training)
        loss = O.keras_bce_from_logits(z, t(target).reshape(z.shape))
        loss.backward()
    finally:
        KBLOCK = old
    return (float(loss.detach()), z.detach().double().numpy(),
            {k: v.grad.detach().double().numpy().copy() for k, v in tp.items()})


NOISE_KBLOCKS = (0, 16, 32, 64)   # 0: one library matmul per product


def noise_band(params: Dict[str, np.ndarray], pos, src, dst, prop, target, mp_steps: int = O.REF_MP_STEPS,
               drop_r=None, drop_o=None, training: bool = True, ref=None):
    """How far valid implementations of the SAME bf16-operand arithmetic land apart on this batch.

    bf16 rounding is discontinuous: an operand that fp32 accumulation order moves across a bf16
    rounding boundary changes by one bf16 ulp (2⁻⁸ relative), which perturbs everything downstream in
    its tower by far more than the fp32 difference that caused it, and the perturbed values cross
    further boundaries (measured: this emulator in fp32 vs fp64 on 64 six-block towers, S = 5 — about
    1 operand in 10⁵ flips in the first layer, yet a third of the logits move, by up to 4.6e-3, and
    the rm.0 kernel gradient by 1.7 % of its norm). No fp32 implementation can therefore match the
    emulator element for element; the engine is held to landing no further from it than other valid
    implementations do. Returns (ref, band): ref = the fp64 emulator's (loss, logits, grads); band =
    per quantity the largest distance from ref over the alternative implementations (fp32 accumulation
    in k-blocks of NOISE_KBLOCKS, like an MFMA k loop, or in one library matmul): {"z_rms", "z_max", "g": {name: relative L2}}."""
    if ref is None:
        ref = loss_and_grads(params, pos, src, dst, prop, target, mp_steps, drop_r, drop_o, training)
    band = {"z_rms": 0.0, "z_max": 0.0, "g": {k: 0.0 for k in ref[2]}}
    for kb in NOISE_KBLOCKS:
        alt = loss_and_grads(params, pos, src, dst, prop, target, mp_steps, drop_r, drop_o, training,
                             dtype=torch.float32, kblock=kb)
        dz = alt[1] - ref[1]
        band["z_rms"] = max(band["z_rms"], float(np.sqrt(np.mean(dz ** 2))))
        band["z_max"] = max(band["z_max"], float(np.abs(dz).max()))
        for k, r in ref[2].items():
            band["g"][k] = max(band["g"][k], rel_l2(alt[2][k], r))
    return ref, band


def rel_l2(a, ref) -> float:
    return float(np.linalg.norm(np.asarray(a, np.float64) - ref) / (np.linalg.norm(ref) + 1e-30))
