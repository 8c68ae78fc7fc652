"""GraphNetwork: the reference's propagation network as a torch module backed by libspwgnn_hip.

Reference graph: src/Networks.py:16-104 (PropagationNetwork.getModel) over the MLP blocks of
src/Blocks.py:12-91. Inputs and output keep the reference layout: objects (B,N,3), sender/receiver
relations (B,N,E), propagation (B,N,100) → per-object stability probability (B,N,1).
"""
from __future__ import annotations

from typing import Dict, Optional

import numpy as np
import torch
from torch import nn

from . import engine as E
from . import params as P
from .batch import TowerBatch


class _PropagationFn(torch.autograd.Function):
    """Forward/backward of the whole graph through the C-ABI; gradients w.r.t. the flat
    parameter buffer and the propagation input."""

    @staticmethod
    def forward(ctx, flat, prop_dummy, batch: TowerBatch, run: E.RunConfig, ws: E.Workspace):
        logits = E.forward(flat, batch, run, ws)
        ctx.batch, ctx.run, ctx.ws = batch, run, ws
        ctx.save_for_backward(flat)
        ctx.want_prop = prop_dummy.requires_grad
        return logits

    @staticmethod
    def backward(ctx, dlogits):
        (flat,) = ctx.saved_tensors
        grads, dprop = E.backward(flat, ctx.batch, ctx.run, ctx.ws, dlogits, want_dprop=ctx.want_prop)
        return grads, dprop, None, None, None


class GraphNetwork(nn.Module):
    """Propagation network (rm, om, rmp, omp) with shared weights across sizes and steps.

    ``mp_steps`` defaults to the reference's 5 (Networks.py:83); ``dropout`` to its 0.1 on the
    two encodings (Networks.py:77-78), active only in training mode.
    """

    def __init__(self, mp_steps: int = E.REF_MP_STEPS, dropout: float = E.REF_DROPOUT, seed: int = 0,
                 device="cuda", params: Optional[Dict[str, np.ndarray]] = None):
        super().__init__()
        self.mp_steps = mp_steps
        self.dropout = dropout
        init = params if params is not None else P.glorot_uniform(seed)
        self.flat = nn.Parameter(P.to_flat(init, device=device))
        self._step_seed = seed * 1000003 + 17

    @property
    def device(self):
        return self.flat.device

    def keras_weights(self) -> Dict[str, np.ndarray]:
        return P.from_flat(self.flat)

    def load_keras_weights(self, params: Dict[str, np.ndarray]):
        with torch.no_grad():
            self.flat.copy_(P.to_flat(params, device=self.flat.device))

    def _run(self) -> E.RunConfig:
        need_grad = torch.is_grad_enabled() and self.flat.requires_grad
        drop = self.training and self.dropout > 0 and need_grad
        seed = 0
        if drop:
            self._step_seed += 1
            seed = self._step_seed
        return E.RunConfig(self.mp_steps, training=need_grad, dropout=self.dropout if drop else 0.0, seed=seed)

    def forward_batch(self, batch: TowerBatch, prop: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Logits (n_nodes,) for a compact batch (the reference returns sigmoid of these)."""
        run = self._run()
        ws = E.Workspace(self.device)
        if prop is not None:
            batch = batch.with_prop(prop)
            # the backward returns dprop as (n_nodes, 100): autograd maps it back through the reshape
            # to whatever layout the caller passed ((B, N, 100) in the reference)
            dummy = prop.reshape(batch.n_nodes, 100)
        else:
            dummy = torch.zeros(0, device=self.device)
        if not run.training:
            with torch.no_grad():
                return E.forward(self.flat.detach(), batch, run, ws)
        return _PropagationFn.apply(self.flat, dummy, batch, run, ws)

    def forward_logits(self, objects, sender_relations, receiver_relations, propagation=None) -> torch.Tensor:
        batch = TowerBatch.from_dense(objects, sender_relations, receiver_relations, None, device=self.device)
        prop = None
        if propagation is not None:
            prop = torch.as_tensor(propagation, dtype=torch.float32, device=self.device).reshape(batch.n_nodes, 100)
        z = self.forward_batch(batch, prop)
        return z.reshape(batch.node_shape)

    def forward(self, objects, sender_relations, receiver_relations, propagation=None) -> torch.Tensor:
        """(B, N, 1) probabilities: sigmoid(x[:, :, :1]) of the last step (Networks.py:93-96)."""
        return torch.sigmoid(self.forward_logits(objects, sender_relations, receiver_relations, propagation))[..., None]

    def forward_pooled(self, objects, sender_relations, receiver_relations, propagation=None,
                       mode: str = "mean_prob") -> torch.Tensor:
        """(B,) per-tower pooled output — the optional GlobalBlock-style readout (not in the
        reference): "mean_prob" / "sum_prob" (Σŷ of JengaBuilder.py:252-256) /
        "mean_logit" / "sum_logit", reduced on device. Inference only (no autograd)."""
        batch = TowerBatch.from_dense(objects, sender_relations, receiver_relations, propagation, device=self.device)
        with torch.no_grad():
            z = E.forward(self.flat.detach(), batch, E.RunConfig(self.mp_steps, training=False), E.Workspace(self.device))
            return E.tower_readout(z, batch, mode)
