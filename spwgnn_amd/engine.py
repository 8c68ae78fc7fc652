"""Thin host wrapper over the C-ABI: workspace management and the per-call entry points.

torch provides device memory (caching allocator) and the current HIP stream; every byte of
arithmetic happens in libspwgnn_hip.so. Nothing here falls back to CPU.
"""
from __future__ import annotations

import ctypes as C
import os
import weakref
from dataclasses import dataclass
from typing import Optional

import torch

from . import _lib, params as P
from .batch import TowerBatch

REF_MP_STEPS = 5       # Networks.py:83
REF_DROPOUT = 0.1      # Networks.py:77-78


def _stream(device: torch.device) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def _require_gpu(t: torch.Tensor, what: str):
    if t.device.type != "cuda":
        raise _lib.SpwgnnError(f"{what} must be a HIP device tensor (got {t.device}); the HIP path has no CPU fallback")


MATH_MODES = {"f32": _lib.MATH_F32, "x6": _lib.MATH_X6, "bf16": _lib.MATH_BF16}


# Replayed steps fold their batch upload and key/step advance into the forward's first launch
# (spwgnn_run.prologue); SPWGNN_NO_PROLOGUE=1 issues them as launches of their own (A/B).
FOLD_PROLOGUE = os.environ.get("SPWGNN_NO_PROLOGUE", "0") in ("", "0")


@dataclass
class RunConfig:
    mp_steps: int = REF_MP_STEPS
    training: bool = False
    dropout: float = 0.0
    seed: int = 0
    math: str = "x6"                     # "x6" split-bf16 matrix products | "f32" f32 MFMA (spwgnn.h)
    prof_kernel: int = 0                 # SPWGNN_K_* to bracket with HIP events (bench only)
    prof_events: Optional[list] = None   # raw hipEvent_t handles, 2 per launch
    seed_dev: Optional[torch.Tensor] = None   # (1,) int64 device word holding the dropout key (replayable steps)
    prologue: Optional["Prologue"] = None      # forward only: a replayed step's upload + key/step advance
    grads_early_event: Optional[torch.cuda.Event] = None   # backward only: spwgnn_run.grads_early_event

    def cstruct(self, with_prologue: bool = False) -> _lib.RunC:
        r = _lib.RunC()
        r.mp_steps = int(self.mp_steps)
        r.training = 1 if self.training else 0
        r.dropout = float(self.dropout)
        r.seed = int(self.seed) & 0xFFFFFFFFFFFFFFFF
        if self.math not in MATH_MODES:
            raise ValueError(f"math must be one of {sorted(MATH_MODES)}")
        r.math = MATH_MODES[self.math]
        if self.prof_kernel and self.prof_events:
            arr = (C.c_void_p * len(self.prof_events))(*self.prof_events)
            self._prof_arr = arr   # keep alive for the call
            r.prof_kernel = int(self.prof_kernel)
            r.prof_count = len(self.prof_events) // 2
            r.prof_events = C.cast(arr, C.c_void_p)
        if self.seed_dev is not None:
            if self.seed_dev.device.type != "cuda" or self.seed_dev.dtype != torch.int64:
                raise ValueError("seed_dev must be a (1,) int64 device tensor")
            r.seed_dev = self.seed_dev.data_ptr()
        if self.grads_early_event is not None:
            h = self.grads_early_event.cuda_event
            if not h:
                raise ValueError("grads_early_event: record the event once first (it has no hipEvent_t yet)")
            r.grads_early_event = h
        if with_prologue and self.prologue is not None:   # spwgnn_forward only
            self._pro_c = self.prologue.cstruct()   # keep alive for the call
            r.prologue = C.cast(C.pointer(self._pro_c), C.c_void_p)
        return r


@dataclass
class Prologue:
    """spwgnn_prologue (include/spwgnn.h): what a replayed step does before its forward, run by the
    forward's first launch instead of two launches of its own — the batch upload (spwgnn_copy_in:
    `nbytes` from the pinned, device-mapped `src_dev_ptr` into `dst`) and the key/step advance
    (spwgnn_step_advance: `key`, `step` device words, `mode` STEP_KEY_*)."""
    dst: Optional[torch.Tensor] = None
    src_dev_ptr: int = 0
    nbytes: int = 0
    key: Optional[torch.Tensor] = None
    step: Optional[torch.Tensor] = None
    mode: int = _lib.STEP_KEY_COUNTER
    seed: int = 0
    rank: int = 0

    def cstruct(self) -> _lib.PrologueC:
        p = _lib.PrologueC()
        if self.nbytes:
            if self.dst is None or not self.src_dev_ptr:
                raise ValueError("prologue copy needs dst and src_dev_ptr")
            _require_gpu(self.dst, "prologue copy destination")
            if self.nbytes > self.dst.numel() * self.dst.element_size():
                raise ValueError("prologue copy beyond its destination")
            p.copy_src, p.copy_dst, p.copy_bytes = int(self.src_dev_ptr), self.dst.data_ptr(), int(self.nbytes)
        if self.key is not None:
            if self.step is None:
                raise ValueError("prologue advance needs key and step words")
            p.key, p.step = self.key.data_ptr(), self.step.data_ptr()
            p.mode, p.seed, p.rank = int(self.mode), int(self.seed) & 0xFFFFFFFFFFFFFFFF, int(self.rank)
        return p


# SPWGNN_POISON_WORKSPACE=1: fill every newly allocated workspace with 0xFF bytes (and the logits,
# gradient and d/d'propagation' outputs with NaN), so a kernel that reads workspace it did not write,
# or leaves part of an output unwritten, turns results into NaN (run the GPU suite with it;
# tests/test_gpu_determinism.py does the same per case)
POISON_WORKSPACE = os.environ.get("SPWGNN_POISON_WORKSPACE", "0") not in ("", "0")


def _poison(t: torch.Tensor) -> torch.Tensor:
    """An output buffer the library must write in full: NaN-filled under SPWGNN_POISON_WORKSPACE."""
    if POISON_WORKSPACE and t.is_floating_point():
        t.fill_(float("nan"))
    return t


class Workspace:
    """Device scratch for one forward (+ its backward). Sized by spwgnn_workspace_bytes."""

    def __init__(self, device):
        self.device = torch.device(device)
        self.buf: Optional[torch.Tensor] = None
        self.fwd_key: Optional[tuple] = None   # what the last forward on this workspace stored
        self.fwd_batch = None                  # weakref to the batch that forward ran on

    @staticmethod
    def key(batch: TowerBatch, run: "RunConfig") -> tuple:
        # sizes and run fields, plus the device arrays the stored activations were computed from:
        # two same-shape batches (equal micro-batches under one seed) must not pass for each other
        return (run.math, int(run.mp_steps), bool(run.training), float(run.dropout), int(run.seed),
                run.seed_dev.data_ptr() if run.seed_dev is not None else 0, batch.n_nodes, batch.n_eblocks, batch.n_wtiles, batch.pos.data_ptr(), batch.edge_src.data_ptr(),
                batch.prop.data_ptr() if batch.prop is not None else 0)

    def holds(self, batch: TowerBatch, run: "RunConfig") -> bool:
        """True when the last forward on this workspace ran `batch` (the same object) with `run`."""
        return (self.buf is not None and self.fwd_batch is not None and self.fwd_batch() is batch
                and self.fwd_key == Workspace.key(batch, run))

    def get(self, nbytes: int) -> torch.Tensor:
        if self.buf is None or self.buf.numel() < nbytes:
            self.buf = None
            self.buf = torch.empty(int(nbytes), dtype=torch.uint8, device=self.device)
            if POISON_WORKSPACE:   # debugging: every fresh workspace byte 0xFF (NaN as fp32)
                self.buf.fill_(0xFF)
        return self.buf


def workspace_bytes(batch: TowerBatch, run: RunConfig) -> int:
    n = int(_lib.lib().spwgnn_workspace_bytes(batch.n_nodes, batch.n_eblocks, run.mp_steps, 1 if run.training else 0))
    if n < 0:
        raise _lib.SpwgnnError("invalid batch shape for workspace")
    return n


def fused_path(batch: TowerBatch, run: RunConfig) -> int:
    """The library's own answer to which launches this batch and run take (spwgnn_fused_path): bit 0 =
    the forward's fused small-batch step loop, bit 1 = the backward's. No device work."""
    b = batch.cstruct()
    r = run.cstruct()
    st = _lib.lib().spwgnn_fused_path(C.byref(b), C.byref(r))
    if st < 0:
        _lib.check(st, "spwgnn_fused_path")
    return int(st)


def team_max_blocks(set_to: Optional[int] = None) -> int:
    """The library's small-batch limit (spwgnn_team_max_blocks): batches of at most this many 32-row
    blocks run the team kernels, larger ones the wide kernels. With ``set_to`` (>= 0) it is changed for
    the process and the previous limit is returned."""
    return int(_lib.lib().spwgnn_team_max_blocks(-1 if set_to is None else int(set_to)))


class wide_kernels:
    """``with wide_kernels(): ...`` — every call inside plans the wide (large-batch) kernels whatever the
    batch size (team limit 0), then the previous limit is restored."""

    def __enter__(self):
        self._prev = team_max_blocks(0)
        return self

    def __exit__(self, *exc):
        team_max_blocks(self._prev)
        return False


def forward(flat_params: torch.Tensor, batch: TowerBatch, run: RunConfig, ws: Workspace,
            logits: Optional[torch.Tensor] = None) -> torch.Tensor:
    _require_gpu(flat_params, "params")
    if flat_params.dtype != torch.float32 or not flat_params.is_contiguous() or flat_params.numel() != P.flat_size():
        raise ValueError("params must be a contiguous fp32 flat buffer of spwgnn_param_count() floats")
    nbytes = workspace_bytes(batch, run)
    buf = ws.get(nbytes)
    if logits is None:
        logits = _poison(torch.empty(batch.n_nodes, dtype=torch.float32, device=batch.device))
    b = batch.cstruct()
    r = run.cstruct(with_prologue=True)
    st = _lib.lib().spwgnn_forward(flat_params.data_ptr(), C.byref(b), C.byref(r), buf.data_ptr(), buf.numel(),
                                   logits.data_ptr(), _stream(batch.device))
    ws.fwd_key = Workspace.key(batch, run) if st == 0 else None
    ws.fwd_batch = weakref.ref(batch) if st == 0 else None
    _lib.check(st, "spwgnn_forward")
    return logits


def backward(flat_params: torch.Tensor, batch: TowerBatch, run: RunConfig, ws: Workspace, dlogits: torch.Tensor,
             grads: Optional[torch.Tensor] = None, want_dprop: bool = False):
    if not run.training:
        raise _lib.SpwgnnError("backward needs a training forward on the same workspace")
    if not ws.holds(batch, run):
        # the backward reads what the forward stored (masks, activations, packed weights); the split-
        # bf16 maths do not store z1/zo1 at all, so a mismatched math or step count reads garbage
        raise _lib.SpwgnnError("backward needs the training forward of the same batch and RunConfig "
                               f"on this workspace (stored {ws.fwd_key}, asked {Workspace.key(batch, run)})")
    dlogits = dlogits.contiguous().to(torch.float32)
    _require_gpu(dlogits, "dlogits")
    if grads is None:
        grads = _poison(torch.empty_like(flat_params))
    dprop = _poison(torch.empty(batch.n_nodes, 100, dtype=torch.float32, device=batch.device)) if want_dprop else None
    b = batch.cstruct()
    r = run.cstruct()
    buf = ws.buf
    st = _lib.lib().spwgnn_backward(flat_params.data_ptr(), C.byref(b), C.byref(r), buf.data_ptr(), buf.numel(),
                                    dlogits.data_ptr(), grads.data_ptr(), dprop.data_ptr() if dprop is not None else None,
                                    _stream(batch.device))
    _lib.check(st, "spwgnn_backward")
    return grads, dprop


def bce_backward(flat_params: torch.Tensor, batch: TowerBatch, run: RunConfig, ws: Workspace, logits: torch.Tensor,
                 targets: torch.Tensor, scratch: "BceScratch", dlogits: Optional[torch.Tensor] = None,
                 total3: Optional[torch.Tensor] = None, weights3: Optional[torch.Tensor] = None,
                 grads: Optional[torch.Tensor] = None, want_dprop: bool = False):
    """bce (or its accumulating form) then backward in one library call (spwgnn_bce_backward, ABI 6):
    bit-identical to the two calls; on the fused small-batch loop the loss needs no launch of its own.
    Returns (out3, dlogits, grads, dprop)."""
    if not run.training:
        raise _lib.SpwgnnError("backward needs a training forward on the same workspace")
    if not ws.holds(batch, run):
        raise _lib.SpwgnnError("backward needs the training forward of the same batch and RunConfig "
                               f"on this workspace (stored {ws.fwd_key}, asked {Workspace.key(batch, run)})")
    targets = targets.reshape(-1).to(torch.float32).contiguous()
    _require_gpu(logits, "logits")
    if dlogits is None:
        dlogits = _poison(torch.empty_like(logits))
    if grads is None:
        grads = _poison(torch.empty_like(flat_params))
    if (total3 is None) != (weights3 is None):
        raise ValueError("total3 and weights3 go together")
    if total3 is not None:
        assert total3.dtype == torch.float64 and weights3.dtype == torch.float64
    dprop = _poison(torch.empty(batch.n_nodes, 100, dtype=torch.float32, device=batch.device)) if want_dprop else None
    b = batch.cstruct()
    r = run.cstruct()
    buf = ws.buf
    st = _lib.lib().spwgnn_bce_backward(
        flat_params.data_ptr(), C.byref(b), C.byref(r), buf.data_ptr(), buf.numel(), logits.data_ptr(),
        targets.data_ptr(), logits.numel(), scratch.out3.data_ptr(), dlogits.data_ptr(), scratch.scratch.data_ptr(),
        weights3.data_ptr() if weights3 is not None else None, total3.data_ptr() if total3 is not None else None,
        grads.data_ptr(), dprop.data_ptr() if dprop is not None else None, _stream(batch.device))
    _lib.check(st, "spwgnn_bce_backward")
    return scratch.out3, dlogits, grads, dprop


class BceScratch:
    def __init__(self, device):
        n = int(_lib.lib().spwgnn_bce_scratch_bytes(1))
        self.scratch = torch.empty(n, dtype=torch.uint8, device=device)
        self.out3 = torch.empty(3, dtype=torch.float32, device=device)


def bce(logits: torch.Tensor, targets: torch.Tensor, scratch: BceScratch, dlogits: Optional[torch.Tensor] = None,
        total3: Optional[torch.Tensor] = None, weights3: Optional[torch.Tensor] = None):
    """Keras binary_crossentropy (+ binary_accuracy numerator) and d loss / d logit on device.
    Returns out3 = [loss, n_correct, n] (device) and dlogits. With total3/weights3 (float64) the
    same launch also does total3 += out3.double() * weights3 (spwgnn_bce_accumulate)."""
    targets = targets.reshape(-1).to(torch.float32).contiguous()
    if dlogits is None:
        dlogits = _poison(torch.empty_like(logits))
    args = (logits.data_ptr(), targets.data_ptr(), logits.numel(), scratch.out3.data_ptr(), dlogits.data_ptr(),
            scratch.scratch.data_ptr())
    if total3 is None:
        st = _lib.lib().spwgnn_bce(*args, _stream(logits.device))
        _lib.check(st, "spwgnn_bce")
    else:
        assert total3.dtype == torch.float64 and weights3 is not None and weights3.dtype == torch.float64
        st = _lib.lib().spwgnn_bce_accumulate(*args, weights3.data_ptr(), total3.data_ptr(), _stream(logits.device))
        _lib.check(st, "spwgnn_bce_accumulate")
    return scratch.out3, dlogits


def adam(params: torch.Tensor, grads: torch.Tensor, m: torch.Tensor, v: torch.Tensor, step: int, lr=5e-4,
         beta1=0.9, beta2=0.999, eps=1e-7, l2=0.0, grad_scale=1.0):
    st = _lib.lib().spwgnn_adam(params.data_ptr(), grads.data_ptr(), m.data_ptr(), v.data_ptr(), params.numel(),
                                int(step), lr, beta1, beta2, eps, l2, grad_scale, _stream(params.device))
    _lib.check(st, "spwgnn_adam")


def adam_dev(params: torch.Tensor, grads: torch.Tensor, m: torch.Tensor, v: torch.Tensor, step_dev: torch.Tensor,
             lr_table: torch.Tensor, beta1=0.9, beta2=0.999, eps=1e-7, l2=0.0, grad_scale=1.0):
    """Adam with the step count read from the device word `step_dev` ((1,) int32) and lr_t from
    `lr_table` (device fp32, built by `adam_lr_table`): capturable into a replayed hipGraph."""
    st = _lib.lib().spwgnn_adam_dev(params.data_ptr(), grads.data_ptr(), m.data_ptr(), v.data_ptr(), params.numel(),
                                    step_dev.data_ptr(), lr_table.data_ptr(), lr_table.numel(), beta1, beta2, eps, l2,
                                    grad_scale, _stream(params.device))
    _lib.check(st, "spwgnn_adam_dev")


def adam_lr_table(n: int, lr=5e-4, beta1=0.9, beta2=0.999, device="cuda") -> torch.Tensor:
    """lr_t of steps 0..n-1 (host-built with spwgnn_adam's own expression), on the device."""
    import numpy as np
    out = np.zeros(int(n), np.float32)
    _lib.check(_lib.lib().spwgnn_adam_lr_table(lr, beta1, beta2, int(n), out.ctypes.data), "spwgnn_adam_lr_table")
    return torch.from_numpy(out).to(device)


def step_advance(key_dev: torch.Tensor, step_dev: torch.Tensor, mode: int = _lib.STEP_KEY_COUNTER, seed: int = 0,
                 rank: int = 0):
    """Start a replayable step on the device: step += 1, dropout key moved on (spwgnn.h)."""
    st = _lib.lib().spwgnn_step_advance(key_dev.data_ptr(), step_dev.data_ptr(), int(mode),
                                        int(seed) & 0xFFFFFFFFFFFFFFFF, int(rank), _stream(key_dev.device))
    _lib.check(st, "spwgnn_step_advance")


def accumulate_out3(total3: torch.Tensor, out3: torch.Tensor, weights3: torch.Tensor) -> None:
    """total3 += out3.double() * weights3 (three float64 sums on the device) in one launch."""
    assert total3.dtype == torch.float64 and weights3.dtype == torch.float64 and out3.dtype == torch.float32
    st = _lib.lib().spwgnn_accumulate_out3(out3.data_ptr(), weights3.data_ptr(), total3.data_ptr(), _stream(out3.device))
    _lib.check(st, "spwgnn_accumulate_out3")


def copy_in(host: torch.Tensor, dev: torch.Tensor, nbytes: int, src_dev_ptr: Optional[int] = None) -> None:
    """dev[:nbytes] ← host[:nbytes] by a kernel on the current stream (spwgnn_copy_in): `host` a pinned
    (device-mapped) tensor, read at `src_dev_ptr` (its device address) when given. Captured into a
    graph it is one kernel node, not a DMA copy."""
    if not host.is_pinned():
        raise ValueError("copy_in reads pinned host memory")
    _require_gpu(dev, "copy_in destination")
    if nbytes > host.numel() * host.element_size() or nbytes > dev.numel() * dev.element_size():
        raise ValueError("copy_in beyond a buffer")
    src = src_dev_ptr if src_dev_ptr is not None else host.data_ptr()
    st = _lib.lib().spwgnn_copy_in(src, dev.data_ptr(), int(nbytes), _stream(dev.device))
    _lib.check(st, "spwgnn_copy_in")


def sigmoid(logits: torch.Tensor) -> torch.Tensor:
    out = torch.empty_like(logits)
    st = _lib.lib().spwgnn_sigmoid(logits.data_ptr(), out.data_ptr(), logits.numel(), _stream(logits.device))
    _lib.check(st, "spwgnn_sigmoid")
    return out


READOUT_MODES = {"sum_prob": _lib.READOUT_SUM_PROB, "mean_prob": _lib.READOUT_MEAN_PROB,
                 "sum_logit": _lib.READOUT_SUM_LOGIT, "mean_logit": _lib.READOUT_MEAN_LOGIT}


def tower_readout(logits: torch.Tensor, batch: TowerBatch, mode: str = "sum_prob") -> torch.Tensor:
    """(T,) per-tower reduction of the node logits on device: "sum_prob" is the Σŷ stability score of
    JengaBuilder.remove_to_demolish (JengaBuilder.py:252-256); "mean_prob" the optional GlobalBlock
    mean pool (not in the reference)."""
    if mode not in READOUT_MODES:
        raise ValueError(f"readout mode must be one of {sorted(READOUT_MODES)}")
    _require_gpu(logits, "logits")
    logits = logits.reshape(-1).contiguous().to(torch.float32)
    if logits.numel() != batch.n_nodes:
        raise ValueError("logits must hold one value per node of the batch")
    out = torch.empty(batch.n_towers, dtype=torch.float32, device=logits.device)
    st = _lib.lib().spwgnn_tower_readout(logits.data_ptr(), batch.tower_offsets.data_ptr(), batch.n_towers,
                                         READOUT_MODES[mode], out.data_ptr(), _stream(logits.device))
    _lib.check(st, "spwgnn_tower_readout")
    return out
