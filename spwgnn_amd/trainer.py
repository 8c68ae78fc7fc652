"""Data-parallel training step: towers sharded over ranks, one RCCL all-reduce of the flat gradient.

The reference trains with Keras fit on one CPU process (src/main.py:92-98; Adam + BCE compiled at
src/Networks.py:101-102). Here every rank owns a shard of the tower batch (towers are independent
graphs, so the shard needs no halo and no data-path collective), runs forward → BCE → backward
through libspwgnn_hip, and the 209,501 fp32 gradients (one flat bucket, 0.84 MB) are summed with
ONE torch.distributed all-reduce (backend "nccl" = RCCL over xGMI on MI355X), then Adam runs on
every rank.

Weighting: the reference's loss is the mean BCE over all B·N nodes of the batch
(src/Networks.py:102). A rank's backward yields the gradient of the mean over ITS nodes, so each
rank scales its gradient by n_local / n_global before the sum; Σ_r (n_r/n)·g_r is then exactly
the gradient of the global mean, for ragged and unequal shards alike (config 4). n_global comes
from the shard plan (`spwgnn_amd/shard.py`) or, when not given, from one 8-byte all-reduce.
Micro-batches (`step` with lists) accumulate their node-weighted gradients before the one
all-reduce and the one Adam update.

The arithmetic engine is pluggable only so the CPU test-suite can drive this control flow under
gloo with the oracle; the product engine is HipEngine and has no CPU fallback.
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.distributed as dist

from . import _lib, engine as E, params as P
from .batch import TowerBatch


_M64 = (1 << 64) - 1


def splitmix64(x: int) -> int:
    """One splitmix64 output step (Steele et al.): a bijective 64-bit mix."""
    x = (x + 0x9E3779B97F4A7C15) & _M64
    x = ((x ^ (x >> 30)) * 0xBF58476D1CE4E5B9) & _M64
    x = ((x ^ (x >> 27)) * 0x94D049BB133111EB) & _M64
    return x ^ (x >> 31)


def dropout_key(seed: int, iteration: int, rank: int, micro: int) -> int:
    """The run's 64-bit dropout key for (seed, optimizer step, rank, micro-batch): each field is
    folded through splitmix64 in turn, so no field overflows into the next (a packed
    ((seed·P + it)·R + rank)·M + micro key collides once rank ≥ R or micro ≥ M)."""
    h = splitmix64(seed & _M64)
    for v in (iteration, rank, micro):
        h = splitmix64(h ^ (v & _M64))
    return h


class HipEngine:
    def __init__(self, device):
        self.device = torch.device(device)
        self.ws = E.Workspace(self.device)
        self.bce_scratch = E.BceScratch(self.device)
        self.grads: Optional[torch.Tensor] = None

    def forward(self, params, batch: TowerBatch, run: E.RunConfig):
        return E.forward(params, batch, run, self.ws)

    def loss(self, logits, target):
        return E.bce(logits, target, self.bce_scratch)

    def backward(self, params, batch, run, dlogits):
        if self.grads is None or self.grads.numel() != params.numel():
            self.grads = torch.empty_like(params)
        g, _ = E.backward(params, batch, run, self.ws, dlogits, grads=self.grads)
        return g

    def early_event(self):
        """The event the library records once the early gradient range is final
        (spwgnn_run.grads_early_event); created (recorded once) on first use."""
        ev = getattr(self, "_early_ev", None)
        if ev is None:
            ev = self._early_ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(self.device))   # creates the underlying hipEvent_t
        return ev

    def adam(self, params, grads, m, v, step, lr, b1, b2, eps, l2, gscale):
        E.adam(params, grads, m, v, step, lr, b1, b2, eps, l2, gscale)


class Trainer:
    """Keras-semantics training step (dropout 0.1, BCE, Adam lr=5e-4 eps=1e-7) with optional DP."""

    def __init__(self, params: torch.Tensor, engine=None, mp_steps: int = E.REF_MP_STEPS,
                 dropout: float = E.REF_DROPOUT, seed: int = 0, lr: float = 5e-4, beta1: float = 0.9,
                 beta2: float = 0.999, eps: float = 1e-7, l2: float = 0.0, group=None, math: str = "x6",
                 buckets: int = 1, overlap: bool = True):
        self.params = params
        self.engine = engine if engine is not None else HipEngine(params.device)
        self.m = torch.zeros_like(params)
        self.v = torch.zeros_like(params)
        self.mp_steps, self.dropout, self.seed, self.math = mp_steps, dropout, seed, math
        self.lr, self.b1, self.b2, self.eps, self.l2 = lr, beta1, beta2, eps, l2
        self.iterations = 0
        self.group = group
        self.distributed = dist.is_available() and dist.is_initialized()
        self.world = dist.get_world_size(group) if self.distributed else 1
        self.rank = dist.get_rank(group) if self.distributed else 0
        self.prof_kernel = 0
        self.prof_events = None
        # gradient all-reduce: `buckets` contiguous 64-float-aligned pieces of the flat gradient, each
        # its own async all-reduce (all in flight together, waited before Adam); ar_events: an optional
        # (start, end) torch.cuda.Event pair recorded around the all-reduce (bench.py's allreduce_ms)
        self.buckets = max(1, int(buckets))
        self.ar_events = None
        # overlap (N > 1, an engine with early_event): the backward records an event once the gradients
        # of the flat range [rmp.1.kernel, end) are final (spwgnn_run.grads_early_event); that range is
        # all-reduced on a side stream while dA, the encoder backward and the encoder-side gradients run
        # (SURVEY §8e), the rest after the backward. ar_early_events: an optional (start, end) event
        # pair recorded on the side stream around the early all-reduce (bench.py's rehearsal trace)
        self.overlap = overlap
        self.ar_early_events = None
        self._side = None
        self._early_lo = next(off for name, off, _ in P.layout() if name == "rmp.1.kernel")
        self._ctr = None          # replayed steps' device counters (replay_body)
        self._ctr_at = 0          # the host iteration count the device step word holds
        self._w3 = {}             # (n_nodes, 1, 1) fp64 weights of a micro-batch's [loss, correct, n]

    def _early(self, run):
        """Overlapped steps: the engine's early-gradient event, handed to the backward through `run`."""
        if not self._split():
            return None
        ev = self.engine.early_event()
        run.grads_early_event = ev
        return ev

    def run_config(self, micro: int = 0) -> E.RunConfig:
        # distinct dropout keys per step, per rank and per micro-batch (different towers)
        key = dropout_key(self.seed, self.iterations, self.rank, micro)
        return E.RunConfig(self.mp_steps, training=True, dropout=self.dropout, seed=key, math=self.math,
                           prof_kernel=self.prof_kernel, prof_events=self.prof_events)

    def _sync_counters(self):
        """Device step word and lr table ← the host's iteration count and (lr, β1, β2), when they
        differ (a step() or an lr change since the last replay)."""
        from .replay import DeviceCounters
        if self._ctr is None:
            self._ctr = DeviceCounters(self.params.device, 0, self.iterations, self.lr, self.b1, self.b2)
        elif self._ctr_at != self.iterations or self._ctr.hyper != (float(self.lr), float(self.b1), float(self.b2)):
            self._ctr.set(step=self.iterations, lr=self.lr, beta1=self.b1, beta2=self.b2)
        self._ctr_at = self.iterations

    def replay_body(self, n_nodes: int, n_global: Optional[int] = None):
        """The launches of one single-batch `step` for spwgnn_amd.replay.ReplayStep (hipGraph
        replay): the dropout key and Adam step are device words (spwgnn_step_advance in the
        Trainer's splitmix key mode, spwgnn_adam_dev), so every replay is the next optimizer step
        with the masks `step` would draw. Single process only (no all-reduce inside a graph).

        Run each step through `replay_step(rs, plan, target)`: a replay advances the device words
        only, and replay_step keeps `iterations` (the host counter `step` reads) in step with them."""
        if self.world > 1:
            raise ValueError("replayed steps are single-process; DP steps use step()")
        if not isinstance(self.engine, HipEngine):
            raise ValueError("replayed steps need the HIP engine")
        self._sync_counters()
        ctr = self._ctr
        w = n_nodes / (n_global or n_nodes)
        grads = torch.empty_like(self.params)

        def body(batch, target, ws, bce, z, dz, pre=None):
            # the key/step advance (and the replayed batch upload, `pre`) ride in the forward's first launch
            pro = None
            if E.FOLD_PROLOGUE:
                pro = pre if pre is not None else E.Prologue()
                pro.key, pro.step, pro.mode, pro.seed, pro.rank = ctr.key, ctr.step, _lib.STEP_KEY_SPLITMIX, self.seed, self.rank
            else:
                E.step_advance(ctr.key, ctr.step, _lib.STEP_KEY_SPLITMIX, self.seed, self.rank)
            run = E.RunConfig(self.mp_steps, training=True, dropout=self.dropout, math=self.math, seed_dev=ctr.key,
                              prologue=pro)
            E.forward(self.params, batch, run, ws, logits=z)
            # the loss and the backward in one call (spwgnn_bce_backward: no loss launch of its own on
            # the fused small-batch loop; bit-identical to bce then backward)
            E.bce_backward(self.params, batch, run, ws, z, target, bce, dlogits=dz, grads=grads)
            if w != 1.0:
                grads.mul_(w)
            E.adam_dev(self.params, grads, self.m, self.v, ctr.step, ctr.lr_table, self.b1, self.b2, self.eps,
                       self.l2)
        return body

    def bucket_bounds(self, n: int):
        """[(start, end)) of the gradient buckets over a flat buffer of n floats (64-float aligned)."""
        k = min(self.buckets, max(1, n // 64))
        cuts = [0] + [min(n, (n * i // k + 63) // 64 * 64) for i in range(1, k)] + [n]
        return [(a, b) for a, b in zip(cuts[:-1], cuts[1:]) if b > a]

    def allreduce(self, acc: torch.Tensor):
        """Σ over ranks of the node-weighted flat gradient (RCCL over xGMI with backend nccl). With
        buckets > 1 the pieces are issued as async all-reduces, all in flight before the first wait."""
        ev = self.ar_events
        if ev is not None:
            ev[0].record()
        if self.buckets == 1:
            dist.all_reduce(acc, op=dist.ReduceOp.SUM, group=self.group)
        else:
            works = [dist.all_reduce(acc[a:b], op=dist.ReduceOp.SUM, group=self.group, async_op=True)
                     for a, b in self.bucket_bounds(acc.numel())]
            for w in works:
                w.wait()
        if ev is not None:
            ev[1].record()

    def _split(self) -> bool:
        # any process group (a one-rank group included: its all-reduce is the identity, the choreography
        # of events, side stream and collectives is the same as at N > 1)
        return self.distributed and self.overlap and hasattr(self.engine, "early_event")

    def _combine(self, acc, g, w, sl, first):
        """acc[sl] ← w·g[sl] (first micro-batch) or acc[sl] + w·g[sl]; acc may be g itself."""
        if first:
            if acc is g:
                if w != 1.0:
                    acc[sl].mul_(w)
            else:
                torch.mul(g[sl], w, out=acc[sl])
        else:
            acc[sl].add_(g[sl], alpha=w)

    def reduce_split(self, acc, g, w, first, ev):
        """The last backward's gradient `g` folded into `acc` (weight w) and the sum over ranks, in two
        pieces: the early range [rmp.1.kernel, end) on a side stream that waits for `ev` (the library
        records it mid-backward), issued before the late range [0, rmp.1.kernel) on the step's stream.
        Elementwise the same arithmetic as `allreduce` after the whole backward."""
        lo = self._early_lo
        early, late = slice(lo, acc.numel()), slice(0, lo)
        cuda = acc.is_cuda
        cur = torch.cuda.current_stream(acc.device) if cuda else None
        if cuda:
            if self._side is None:
                # high priority: a stream of its own on the device's hardware queues, so its wait on the
                # mid-backward event is not queued behind the step stream's remaining kernels
                self._side = torch.cuda.Stream(acc.device, priority=-1)
            self._side.wait_event(ev)
            ctx = torch.cuda.stream(self._side)
        else:
            import contextlib
            ctx = contextlib.nullcontext()
        with ctx:
            if self.ar_early_events is not None:
                self.ar_early_events[0].record()
            self._combine(acc, g, w, early, first)
            work = dist.all_reduce(acc[early], op=dist.ReduceOp.SUM, group=self.group, async_op=True)
            if self.ar_early_events is not None:   # timing: the side stream waits for the early piece
                work.wait()
                self.ar_early_events[1].record()
        self._combine(acc, g, w, late, first)
        if self.ar_events is not None:
            self.ar_events[0].record()
        dist.all_reduce(acc[late], op=dist.ReduceOp.SUM, group=self.group)
        work.wait()   # the step's stream (CUDA) / the host (CPU tensors) waits for the early piece
        if cuda:
            cur.wait_stream(self._side)
        if self.ar_events is not None:
            self.ar_events[1].record()

    def replay_step(self, rs, plan, target):
        """One replayed optimizer step (rs: a ReplayStep/ReplayCache over `replay_body`): the
        device words are first brought to the host's counters (a `step()` may have run in
        between), the step runs, and the host counter advances with the device one."""
        self._sync_counters()
        out = rs(plan, target)
        self.iterations += 1
        self._ctr_at = self.iterations
        return out

    def step(self, batch, target, n_global: Optional[int] = None):
        """One optimizer step. `batch`/`target` may be lists (micro-batches of this rank's shard);
        `n_global` = nodes in the whole global batch (all ranks, all micro-batches). Returns one
        [loss, correct, n] device tensor for this rank's shard: the node-weighted mean BCE over its
        micro-batches, the binary_accuracy numerator and the node count."""
        batches = batch if isinstance(batch, (list, tuple)) else [batch]
        targets = target if isinstance(target, (list, tuple)) else [target]
        if len(batches) != len(targets) or not batches:
            raise ValueError("one target per micro-batch")
        n_local = sum(b.n_nodes for b in batches)
        if n_global is None:
            n_global = n_local
            if self.world > 1:
                t = torch.tensor([float(n_local)], dtype=torch.float64,
                                 device=self.params.device if dist.get_backend(self.group) != "gloo" else "cpu")
                dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group)
                n_global = int(t.item())
        run = self.run_config()
        acc = None
        tot3 = None
        if len(batches) == 1:   # one batch: its [loss, correct, n] as the engine computed them (one copy)
            b, tg = batches[0], targets[0]
            z = self.engine.forward(self.params, b, run)
            out3, dz = self.engine.loss(z, tg)
            res = out3.clone()          # the engine reuses its out3 buffer
            ev = self._early(run)
            acc = self.engine.backward(self.params, b, run, dz)
            w = b.n_nodes / n_global
            if ev is not None:
                self.reduce_split(acc, acc, w, True, ev)
            else:
                if w != 1.0:
                    acc.mul_(w)
                if self.distributed:   # any process group (one rank: the identity, through the collective)
                    self.allreduce(acc)
            self.iterations += 1
            self.engine.adam(self.params, acc, self.m, self.v, self.iterations, self.lr, self.b1, self.b2, self.eps,
                             self.l2, 1.0)
            return res.float() if res.dtype != torch.float32 else res
        for i, (b, tg) in enumerate(zip(batches, targets)):
            if i:
                run = self.run_config(micro=i)
            z = self.engine.forward(self.params, b, run)
            out3, dz = self.engine.loss(z, tg)
            # [loss, correct, n] of this micro-batch, folded in before the engine reuses its buffer:
            # Σ loss_i·n_i, Σ correct_i, Σ n_i (the engine's out3 is one persistent tensor)
            key = (b.n_nodes, out3.device)
            wt = self._w3.pop(key, None)
            if wt is None:
                wt = out3.new_tensor([float(b.n_nodes), 1.0, 1.0], dtype=torch.float64)
            self._w3[key] = wt            # most recent last; ragged micro-batches keep at most 16
            while len(self._w3) > 16:
                self._w3.pop(next(iter(self._w3)))
            w3 = out3.double() * wt
            tot3 = w3 if tot3 is None else tot3 + w3
            last = i == len(batches) - 1
            ev = self._early(run) if last else None
            g = self.engine.backward(self.params, b, run, dz)
            w = b.n_nodes / n_global
            if ev is not None:   # the last micro-batch: accumulate and reduce in two pieces
                if acc is None:
                    if getattr(self, "_acc", None) is None or self._acc.shape != g.shape or self._acc.device != g.device:
                        self._acc = torch.empty_like(g)
                    acc = self._acc
                    self.reduce_split(acc, g, w, True, ev)
                else:
                    self.reduce_split(acc, g, w, False, ev)
                continue
            if acc is None:
                # the engine writes every backward into one buffer (HipEngine.grads), so the sum lives in
                # a buffer of its own: the Trainer's persistent accumulator, overwritten here
                if getattr(self, "_acc", None) is None or self._acc.shape != g.shape or self._acc.device != g.device:
                    self._acc = torch.empty_like(g)
                acc = torch.mul(g, w, out=self._acc)
            else:
                acc.add_(g, alpha=w)
        if self.distributed and not self._split():
            self.allreduce(acc)
        self.iterations += 1
        self.engine.adam(self.params, acc, self.m, self.v, self.iterations, self.lr, self.b1, self.b2, self.eps,
                         self.l2, 1.0)
        # node-weighted mean loss of this rank's shard, total correct, total nodes (device, fp32)
        return torch.stack([tot3[0] / tot3[2], tot3[1], tot3[2]]).float()
