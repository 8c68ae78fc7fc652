#!/usr/bin/env python3
"""Benchmark: towers/s of the propagation-network hot path on MI355X, per BASELINE.json config.

Default (the headline metric): one full training step (forward + BCE + backward [+ RCCL
all-reduce] + Adam) on synthetic 6-block Jenga towers, 65,536 towers per GPU, 5 propagation steps,
dropout 0.1, fp32-class (x6) arithmetic. `--config K` runs BASELINE.json configs[K-1] instead:

  1  6-block towers, 32 per batch, S=1, thresholded relations (the reference's CPU path; the GPU
     step is launch-bound at this size — the line exists so the CPU baseline has its GPU twin)
  2  6-block towers, 4,096 per GPU, S=3, thresholded relations, fp32-class (x6)
  3  12-block fully connected towers, 65,536 per GPU, S=5, bf16 arithmetic
  4  ragged 4–16-block towers, 2^20 over 8 GPUs = 131,072 per GPU trained as 2 micro-batches of
     65,536, thresholded relations, S=5, bf16 arithmetic
  5  32-block fully connected towers, 8,192 per GPU, S=10, forward only, hipGraph replay

Contract: `python bench.py --gpus N --steps K --warmup W` (N>1 under torch.distributed.run, one
rank per GPU). Prints ONE JSON line on rank 0. See DESIGN.md §7 for the roofline accounting.
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from spwgnn_amd import _lib, params as P  # noqa: E402
from spwgnn_amd import data as D  # noqa: E402
from spwgnn_amd.batch import HostPlan, TowerBatch  # noqa: E402
from spwgnn_amd.trainer import Trainer  # noqa: E402

METRIC = "towers/sec fwd+bwd, 6-block batch=65k, 1/2/4/8 MI355X; achieved HBM GB/s"
PEAK_FP32_TFLOPS = 157.3    # MI355X_MICROARCH.md: fp32 MFMA (= vector) peak
PEAK_BF16_TFLOPS = 2500.0   # MI355X_MICROARCH.md: dense bf16 MFMA peak
PEAK_HBM_GBS = 8000.0
# x6 math runs each fp32 product as 6 bf16 MFMA products: its fp32-equivalent matrix peak
PEAK_X6_TFLOPS = PEAK_BF16_TFLOPS / 6
MATH_PEAK = {"x6": PEAK_X6_TFLOPS, "f32": PEAK_FP32_TFLOPS, "bf16": PEAK_BF16_TFLOPS}
PEAK_NOTE = {"x6": "x6: fp32 products as 6 bf16 MFMA products, peak = 2.5 PF bf16 / 6",
             "f32": "f32 MFMA peak 157.3 TF", "bf16": "bf16 MFMA dense peak 2.5 PF"}
MATH_DESC = {"x6": "x6: each fp32 matrix product as 6 bf16 MFMA products of 3-way split operands, fp32 "
                   "accumulation (DESIGN.md §3b)", "f32": "f32 MFMA",
             "bf16": "bf16: operands rounded to bf16, one bf16 MFMA product, fp32 accumulation"}

# BASELINE.json configs (index = position + 1; 0 = the headline metric's configuration)
CONFIGS = {
    0: dict(nodes=6, towers=65536, S=5, math="x6", relations="full", mode="train"),
    1: dict(nodes=6, towers=32, S=1, math="x6", relations="threshold", mode="train", replay=True),
    2: dict(nodes=6, towers=4096, S=3, math="x6", relations="threshold", mode="train"),
    3: dict(nodes=12, towers=65536, S=5, math="bf16", relations="full", mode="train"),
    4: dict(nodes=(4, 16), towers=131072, S=5, math="bf16", relations="threshold", mode="train", micro=65536),
    5: dict(nodes=32, towers=8192, S=10, math="x6", relations="full", mode="infer"),
}

# algorithmic FLOPs PER STEP of each timed kernel, as f(real edges, nodes, S); the
# launches per step are counted from the HIP events the library recorded, so a kernel family (the
# k_wgrad_ws weight gradients: 12 launches of different shapes) reports FLOPs and time per step
def _wgrad_ws_flops(Ne, Nn, S):
    """the stored-operand weight gradients (k_wgrad_ws, split-bf16 maths): rm.1-3 and W1a over the
    edges ([z | 1]ᵀ·dz, 151×150 each), W1b/W1c (100×150), W3 ([H2s | deg]ᵀ·g, 151×100), omp.0's a and
    P parts (100×100) and omp.1 ([o1 | 1]ᵀ·dx, 101×101) over nodes × steps, omp.0's c_o part on Σ_s do1
    and om.1 (101×100 each) over the nodes"""
    return 2.0 * (4 * 151 * 150 * Ne + S * Nn * (2 * 100 * 150 + 151 * 100 + 2 * 100 * 100 + 101 * 101)
                  + Nn * 2 * 101 * 100)


KERNELS = {
    "edge_fwd": (_lib.K_EDGE_FWD, lambda Ne, Nn, S: 2.0 * 150 * 150 * Ne * S),
    "edge_bwd": (_lib.K_EDGE_BWD, lambda Ne, Nn, S: 2.0 * 150 * 150 * Ne * S),
    "node_fwd": (_lib.K_NODE_FWD, lambda Ne, Nn, S: 2.0 * (151 * 100 + 300 * 100 + 100 * 101 + 2 * 100 * 150) * Nn * S),
    "node_bwd": (_lib.K_NODE_BWD, lambda Ne, Nn, S: 2.0 * (2 * 150 * 100 + 101 * 100 + 300 * 100 + 150 * 100) * Nn * S),
    "wgrad_w2": (_lib.K_WGRAD_W2, lambda Ne, Nn, S: 2.0 * 151 * 150 * Ne * S),
    "wgrad_ws": (_lib.K_WGRAD_WS, _wgrad_ws_flops),
    "dA": (_lib.K_DA, lambda Ne, Nn, S: 2.0 * 150 * 150 * Ne * S),
    "enc_edge": (_lib.K_ENC_EDGE, lambda Ne, Nn, S: 2.0 * (2 * 150 + 4 * 150 * 150) * Ne),
    "enc_edge_bwd": (_lib.K_ENC_EDGE_BWD, lambda Ne, Nn, S: 2.0 * 4 * 150 * 150 * Ne),
    "enc_node": (_lib.K_ENC_NODE, lambda Ne, Nn, S: 2.0 * (2 * 100 + 100 * 100 + 2 * 100 * 150) * Nn),
    "enc_node_bwd": (_lib.K_ENC_NODE_BWD, lambda Ne, Nn, S: 2.0 * 2 * 100 * 100 * Nn),
}
INFER_KERNELS = ("edge_fwd", "node_fwd", "enc_edge", "enc_node")
# Small batches (≤ kTeamMaxBlocks wave-tiles and blocks, ≤ 16-node tiles, split-bf16 math) run the
# fused launches, each timed under one id: its FLOPs are those of the phases it holds,
# its PMC summary rows those of the fused kernel
FUSED_PARTS = {"edge_fwd": ("edge_fwd", "node_fwd"), "node_bwd": ("node_bwd", "edge_bwd"),
               "enc_edge_bwd": ("dA", "enc_edge_bwd", "enc_node_bwd"), "enc_edge": ("enc_edge", "enc_node"),
               "wgrad_ws": ("wgrad_ws", "wgrad_w2")}
FUSED_PMC = {"edge_fwd": "k_fwd_fused", "node_bwd": "k_bwd_fused", "enc_edge_bwd": "k_bwd_enc_pair",
             "enc_edge": "k_enc_pair", "wgrad_ws": "k_wgrad_ws"}
_FUSED = [False]


def fused_small(batches, math, S, dropout=0.1) -> bool:
    """Whether these batches' training steps take the fused small-batch launches: the
    library's own gate (spwgnn_fused_path), so the kernel table's attribution cannot drift from it."""
    from spwgnn_amd import engine as E
    run = E.RunConfig(S, training=True, dropout=dropout, math=math)
    return all(E.fused_path(b, run) == 3 for b in batches)


def kernel_flops(kernel, Ne, Nn, S):
    parts = FUSED_PARTS.get(kernel, (kernel,)) if _FUSED[0] else (kernel,)
    return sum(KERNELS[k][1](Ne, Nn, S) for k in parts)
MAX_LAUNCHES = 32      # event pairs reserved per kernel per micro-batch and step (the family has 12)
# device kernel name prefix in the rocprofv3 PMC summaries (tools/pmcsum.py)
PMC_PREFIX = {"edge_fwd": "k_edge_fwd", "edge_bwd": "k_edge_bwd", "node_fwd": "k_node_fwd",
              "node_bwd": "k_node_bwd", "wgrad_w2": "k_w2grad", "enc_edge": "k_enc_edge", "dA": "k_dA",
              "enc_edge_bwd": "k_enc_edge_bwd", "wgrad_ws": "k_wgrad_ws", "enc_node": "k_enc_node",
              "enc_node_bwd": "k_enc_node_bwd"}


def fwd_flops(Ne: int, Nn: int, S: int) -> float:
    """Forward FLOPs as the kernels compute them (rmp layer 3 behind the receiver sum)."""
    return 2.0 * (Ne * (2 * 150 + 4 * 150 * 150) + Nn * (2 * 100 + 100 * 100)
                  + S * (Ne * 150 * 150 + Nn * (151 * 100 + 300 * 100 + 100 * 101 + 2 * 100 * 150))
                  - Nn * 2 * 100 * 150)


def step_flops(Ne: int, Nn: int, S: int) -> float:
    """Algorithmic FLOPs of one fwd+bwd training step in the form the kernels compute."""
    bwd_edge = Ne * (4 * 150 * 150 + 4 * 151 * 150 + 3 * 100) + S * Ne * (150 * 150 + 151 * 150)
    bwd_node = Nn * (100 * 100 + 101 * 100 + 3 * 100) + S * Nn * (
        2 * 150 * 100 + 101 * 100 + 300 * 100 + 150 * 100     # activation grads
        + 2 * 100 * 150 + 151 * 100 + 301 * 100 + 101 * 101)  # weight grads
    return fwd_flops(Ne, Nn, S) + 2.0 * (bwd_edge + bwd_node)


class HipEvents:
    def __init__(self, n):
        self.hip = _lib.hip_runtime()   # the runtime torch and the library run on
        self.ev = []
        for _ in range(n):
            e = C.c_void_p()
            if self.hip.hipEventCreate(C.byref(e)) != 0:
                raise RuntimeError("hipEventCreate failed")
            self.ev.append(e.value)

    def elapsed_ms(self, a, b) -> float:
        ms = C.c_float()
        s1 = self.hip.hipEventSynchronize(C.c_void_p(self.ev[b]))
        st = self.hip.hipEventElapsedTime(C.byref(ms), C.c_void_p(self.ev[a]), C.c_void_p(self.ev[b]))
        if st != 0 or s1 != 0:
            # a pair the library did not record: HIP keeps the failure as the thread's last error,
            # which the library's next launch check (hipGetLastError) would report as its own — clear it
            self.hip.hipGetLastError()
            raise RuntimeError(f"hipEventElapsedTime failed ({st})")
        return ms.value

    def close(self):
        for e in self.ev:
            self.hip.hipEventDestroy(C.c_void_p(e))


# ------------------------------------------------------------------------------ workloads
PACK_OFF = os.environ.get("SPWGNN_NO_PACK", "0") not in ("", "0")   # A/B: ragged towers in input order
NW_MAX = int(os.environ.get("SPWGNN_NW_MAX", "0")) or None           # A/B: nodes per wave-tile (default plan)


def make_workload(cfg: dict, rank: int, device, world: int = 1, plans: bool = False):
    """This rank's part of the job's synthetic global batch and its targets.

    Every rank builds the same global batch of towers·world towers from one seed, cuts it with the
    cost planner `shard.plan_shards` (contiguous tower ranges of near-equal algorithmic cost; equal
    ranges for uniform towers) and keeps its own range, as micro-batches when the config has them.
    Returns (batches, targets, n_global): n_global = nodes in the whole global batch, taken from the
    plan, so the Trainer needs no per-step all-reduce of node counts. `plans`: host plans sized for
    every relation slot (replayed steps, spwgnn_amd/replay.py) and host targets instead."""
    from spwgnn_amd import shard
    B, S = cfg["towers"] * world, cfg["S"]
    thr = D.RELATION_THRESHOLD if cfg["relations"] == "threshold" else None
    ragged = isinstance(cfg["nodes"], tuple)
    if ragged:                                     # config 4: ragged towers
        lo, hi = cfg["nodes"]
        pos, sizes, src, dst, te, _ = D.ragged_batch(B, lo, hi, seed=4000, threshold=thr)
    else:
        N = cfg["nodes"]
        raw = D.synthetic_towers_fast(B, N, seed=1000 + 97 * N)
        sizes = np.full(B, N, np.int32)
        m_idx, j_idx = np.nonzero(~np.eye(N, dtype=bool))           # sender-major slots (main.py:72-81)
        keep = np.ones((B, len(m_idx)), bool) if thr is None else \
            np.linalg.norm(raw[:, m_idx, 0:2] - raw[:, j_idx, 0:2], axis=2) < thr
        tt, kk = np.nonzero(keep)
        src = (tt * N + m_idx[kk]).astype(np.int32)
        dst = (tt * N + j_idx[kk]).astype(np.int32)
        te = keep.sum(axis=1).astype(np.int32)
        pos = (raw / D.RELATION_THRESHOLD).astype(np.float32).reshape(B * N, 3)
    off = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
    n_global = int(off[-1])
    target_all = np.random.default_rng(17).integers(0, 2, size=n_global).astype(np.float32)
    a, b = shard.plan_shards(sizes, te, world, mp_steps=S)[rank]
    batches, targets = [], []
    for x, y in shard.micro_batches(a, b, cfg.get("micro") or max(b - a, 1)):
        part = D.edge_slice(pos, sizes, src, dst, te, x, y)
        if plans:
            batches.append(HostPlan.build(*part, edge_cap=part[1] * (part[1] - 1)))
            targets.append(target_all[off[x]:off[y]])
            continue
        # ragged towers: planned in spwgnn_plan_order's order (67 % → 78 % block fill at config 4); the
        # targets follow the plan's node order (the loss is a mean over nodes: order-free)
        bt = TowerBatch.from_edges(*part, nw_max=NW_MAX, device=device, pack=ragged and not PACK_OFF)
        batches.append(bt)
        targets.append(torch.tensor(bt.to_plan_order(target_all[off[x]:off[y]]), device=device))
    return batches, targets, n_global


def workload_name(cfg: dict, world: int, dropout: float) -> str:
    N = cfg["nodes"]
    nd = f"{N[0]}-{N[1]}-block ragged" if isinstance(N, tuple) else f"{N}-block"
    rel = "fully connected" if cfg["relations"] == "full" else "thresholded relations (raw distance < 170)"
    if cfg["mode"] == "infer":
        return f"forward, {nd} towers {rel}, {cfg['towers']} towers/GPU, {cfg['S']} MP steps, hipGraph replay"
    mb = f" as micro-batches of {cfg['micro']}" if cfg.get("micro") else ""
    return (f"train step fwd+BCE+bwd+{'allreduce+' if world > 1 else ''}Adam, {nd} towers {rel}, "
            f"{cfg['towers']} towers/GPU{mb}, {cfg['S']} MP steps, dropout {dropout}, {cfg['math']} math")


# ------------------------------------------------------------------------------ CPU baseline
def cpu_sample(cfg: dict, n_sample: int):
    """A bounded sample of the config's towers for the oracle: (objects, Rs, Rr) groups of equal N."""
    N = cfg["nodes"]
    thr = D.RELATION_THRESHOLD if cfg["relations"] == "threshold" else None
    if isinstance(N, tuple):
        pos, sizes, src, dst, te, raw = D.ragged_batch(n_sample, N[0], N[1], seed=77, threshold=thr)
        groups = []
        for n in np.unique(sizes):
            r = np.stack([raw[t] for t in np.nonzero(sizes == n)[0]])
            groups.append(((r / D.RELATION_THRESHOLD).astype(np.float32),) + D.relation_matrices(r, thr))
        return groups
    raw = D.synthetic_towers(n_sample, N, seed=123)
    return [((raw / D.RELATION_THRESHOLD).astype(np.float32),) + D.relation_matrices(raw, thr)]


def cpu_time(cfg: dict, seconds: float, threads: int, form: str):
    """The oracle (torch-CPU restatement of Networks.py, fp32 like Keras floatx) on a bounded sample:
    fwd+bwd for training configs, forward only for inference; `form` = "dense" (the literal one-hot
    bmm graph Keras executes) or "gather" (index gather + index_add)."""
    from oracle import model as O
    torch.set_num_threads(threads)
    S = cfg["S"]
    infer = cfg["mode"] == "infer"
    n_sample = 16 if infer else (64 if cfg["nodes"] in (12,) or isinstance(cfg["nodes"], tuple) else 256)
    n_sample = min(n_sample, cfg["towers"])
    groups = cpu_sample(cfg, n_sample)
    p = O.to_torch(O.glorot_uniform_params(0), dtype=torch.float32, requires_grad=not infer)
    prepared = []
    for obj, Rs, Rr in groups:
        B, N = obj.shape[:2]
        t = torch.tensor(np.random.default_rng(0).integers(0, 2, size=(B, N)).astype(np.float32))
        if form == "dense":
            args = tuple(torch.tensor(a, dtype=torch.float32) for a in (obj, Rs, Rr)) + (torch.zeros(B, N, 100),)
        else:
            e = np.array(O.dense_to_edges(Rs, Rr), np.int64).reshape(-1, 4)   # (tower, slot, sender, receiver)
            args = (torch.tensor(obj.reshape(B * N, 3)), torch.as_tensor(e[:, 0] * N + e[:, 2]),
                    torch.as_tensor(e[:, 0] * N + e[:, 3]), torch.zeros(B * N, 100))
        prepared.append((args, t))

    def one():
        for args, t in prepared:
            if infer:
                with torch.no_grad():
                    (O.forward_dense if form == "dense" else O.forward_gather)(p, *args, S)
                continue
            for v in p.values():
                v.grad = None
            z = (O.forward_dense if form == "dense" else O.forward_gather)(p, *args, S)
            O.keras_bce_from_logits(z.reshape(t.shape), t).backward()

    one()
    n, t0 = 0, time.perf_counter()
    while True:
        one()
        n += 1
        el = time.perf_counter() - t0
        if (el > seconds and n >= 3) or n >= 500:
            break
    return n_sample * n / el, f"{n_sample} towers x {n} iters, {el:.1f}s"


def usable_cores():
    """(cores this process can actually run on, affinity count, cgroup CPU quota or None): the affinity
    set (len(os.sched_getaffinity(0))) capped by the cgroup's CPU quota (cpu.max) and by
    OMP_NUM_THREADS when the environment declares its share that way. On a shared box the affinity
    set lists the whole machine; oversubscribing torch's thread pool there made one run of the oracle
    take minutes instead of seconds."""
    aff = max(1, len(os.sched_getaffinity(0)))
    quota = None
    for path in ("/sys/fs/cgroup/cpu.max",):
        try:
            q, per = open(path).read().split()[:2]
            if q != "max":
                quota = max(1, -(-int(q) // int(per)))
        except (OSError, ValueError):
            pass
    if quota is None:
        try:   # cgroup v1
            q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
            per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
            if q > 0:
                quota = max(1, -(-q // per))
        except (OSError, ValueError):
            pass
    cores = min(aff, quota) if quota else aff
    # the box's declared share (gpurun sets OMP_NUM_THREADS to the CPUs a one-GPU job may use)
    env = os.environ.get("OMP_NUM_THREADS", "")
    if env.isdigit() and int(env) > 0:
        cores = min(cores, int(env))
    return cores, aff, quota


def cpu_baseline(cfg: dict, seconds: float):
    """SURVEY §8d / BASELINE.md CPU plan: the oracle on every host core this process can use (the
    affinity set, capped by the cgroup's CPU quota; the reported value: the literal dense form Keras
    runs), its gather form on the same cores, and beside them the dense form at 16 threads and at 1."""
    threads, aff, quota = usable_cores()
    print(f"cpu_baseline: {threads} threads (affinity {aff}, cgroup quota {quota})", file=sys.stderr, flush=True)
    dense, dsamp = cpu_time(cfg, seconds, threads, "dense")
    print(f"cpu_baseline: dense {dense:.1f} towers/s", file=sys.stderr, flush=True)
    gather, gsamp = cpu_time(cfg, seconds / 2, threads, "gather")
    t16 = min(16, threads)
    d16, samp16 = (dense, dsamp) if t16 == threads else cpu_time(cfg, seconds / 2, t16, "dense")
    one, osamp = cpu_time(cfg, max(3.0, seconds / 4), 1, "dense")
    what = "fwd" if cfg["mode"] == "infer" else "fwd+bwd"
    return {"value": round(dense, 1), "unit": "towers/s", "cores": threads, "affinity_cores": aff,
            "cgroup_cpu_quota": quota, "kind": "port",
            "sample": f"oracle.forward_dense fp32 {what} ({dsamp}), N={cfg['nodes']}, S={cfg['S']}, "
                      f"{cfg['relations']} relations, torch CPU threads={threads} (affinity {aff}, cgroup quota {quota}); gather "
                      f"form {gather:.1f} towers/s ({gsamp}); dense at {t16} threads {d16:.1f} towers/s "
                      f"({samp16}); dense at 1 thread {one:.1f} towers/s ({osamp})",
            "value_gather": round(gather, 1), "value_16threads": round(d16, 1), "value_1thread": round(one, 1)}


# ------------------------------------------------------------------------------ PMC traffic
def pmc_path(config: int) -> str:
    return os.path.join(ROOT, "profiles", "pmc_summary.json" if config == 0 else f"pmc_summary_config{config}.json")


def load_pmc(config: int, kernel: str, math: str, workload: str):
    """HBM bytes per launch of `kernel` (FETCH_SIZE x2 gfx950 correction + WRITE_SIZE, averaged over
    the launches of every variant of that kernel) from the committed rocprofv3 summary of this
    config, or None when absent or collected on another workload."""
    path = pmc_path(config)
    if not os.path.exists(path):
        return None
    try:
        with open(path) as f:
            d = json.load(f)
        meta = d.get("_workload", {})
        if meta and (meta.get("workload") != workload or meta.get("math") != math):
            return None
        tot = cnt = 0.0
        prefix = FUSED_PMC.get(kernel, PMC_PREFIX[kernel]) if _FUSED[0] else PMC_PREFIX[kernel]
        for name, v in d.items():
            if kernel in ("enc_edge", "enc_node") and name.startswith(PMC_PREFIX[kernel] + "_bwd"):
                continue
            if name.startswith(prefix) and "hbm_read_bytes" in v and "hbm_write_bytes" in v:
                tot += (v["hbm_read_bytes"] + v["hbm_write_bytes"]) * v["dispatches"]
                cnt += v["dispatches"]
        return tot / cnt if cnt else None
    except Exception:
        return None


def step_hbm(config: int, ms_per_step: float, math: str, workload: str):
    """Whole-step HBM bytes from the committed PMC summary of this config (mean bytes per dispatch ×
    dispatches, over the steps of that profiling run), divided by THIS run's step time."""
    path = pmc_path(config)
    if not os.path.exists(path):
        return None
    try:
        with open(path) as f:
            d = json.load(f)
        meta = d.get("_workload", {})
        if meta and (meta.get("workload") != workload or meta.get("math") != math):
            return None
        # one Adam per training step; one weight prep per forward (inference replays)
        steps = meta.get("steps") or d.get("k_adam", {}).get("dispatches", 0) or \
            d.get("k_prep", {}).get("dispatches", 0) or d.get("k_prep_weights", {}).get("dispatches", 0)
        if not steps:
            return None
        tot = sum(v.get("hbm_read_bytes", 0.0) * v["dispatches"] + v.get("hbm_write_bytes", 0.0) * v["dispatches"]
                  for v in d.values() if isinstance(v, dict) and "dispatches" in v)
        per = tot / steps
        gbs = per / (ms_per_step * 1e-3) / 1e9
        return {"bytes_per_step": round(per), "achieved_gbs": round(gbs, 1), "peak_gbs": PEAK_HBM_GBS,
                "frac": round(gbs / PEAK_HBM_GBS, 4),
                "source": f"{os.path.relpath(path, ROOT)}: rocprofv3 FETCH_SIZE x2 + WRITE_SIZE per kernel from a "
                          "separate profiling run of this workload, divided by this run's step time"}
    except Exception:
        return None


# Algorithmic (compulsory) HBM bytes PER STEP of each timed kernel: every array it must read or write,
# once, real rows and real features only (150-wide edge/node-message rows, 100-wide state rows; an
# fp32 element is 4 B, a bf16-stored operand 2 B — bf16 math's §3g/§3o arrays and U, V (§3ze) — h1>0 / h2>0 words 19 B
# per edge each. Not the measured traffic (`traffic`, PMC); the roofline picks the roof whose floor
# (bytes ÷ 8 TB/s or FLOPs ÷ matrix peak) is the larger — the kernel's arithmetic intensity against
# the ridge point.
def kernel_bytes(kernel, Ne, Nn, S, math):
    F, W, WN, MK = 4.0, 150, 100, 19.0
    B = 2.0 if math == "bf16" else F          # operand-only arrays stored as bf16 in bf16 math
    edge = {
        "edge_fwd": S * (Ne * (W * B + 2 * MK) + Nn * (2 * W * B + (W + 1) * B)),
        "edge_bwd": S * (Ne * 2 * MK + Nn * (W * F + 2 * W * B)),
        "dA": Ne * (S * 2 * MK + W * B) + S * Nn * W * F,
        "wgrad_w2": Ne * W * B + S * (Ne * 2 * MK + Nn * (2 * W * B + W * F)),
        "node_fwd": S * Nn * ((W + 1) * B + 2 * WN * F + WN * F + WN * B + WN * F + 2 * W * B),
        "node_bwd": S * Nn * (2 * WN * F + WN * B + 2 * W * B + WN * B + W * F + 2 * WN * F + WN * B),
        "enc_edge": Ne * (16 + 8 + 4 * W * B + 4 * MK),
        "enc_edge_bwd": Ne * (W * B + 4 * MK + 4 * W * B),
        "enc_node": Nn * (16 + WN * F + 2 * W * B + 2 * MK),
        "enc_node_bwd": Nn * (S * WN * F + 3 * WN * F),
        # the weight gradients' X and Y operands: rm.1 (X rebuilt from the 8-B d), rm.2, rm.3, W1a per
        # edge; W1b, W1c, omp.0 P/a parts, omp.1, W3 per node·step; omp.0 c part and om.1 per node
        "wgrad_ws": Ne * (8 + W * B + 3 * 2 * W * B) + S * Nn * (2 * (WN * F + W * B) + 2 * (WN * F + WN * F)
                                                                  + 2 * WN * B + (W + 1) * B + WN * B)
                    + Nn * (2 * WN * F + 8 + WN * F),
    }
    return edge.get(kernel)


def roofline(kernel: str, kern_ms, launches_per_step, Ne, Nn, S, math, config, workload):
    """A timed kernel's roofline. Both floors of one launch: its algorithmic FLOPs ÷ the matrix peak of
    the math it runs in, and its algorithmic bytes (kernel_bytes) ÷ 8 TB/s; `bound` is the roof with
    the larger floor (the kernel's arithmetic intensity against the ridge point), `achieved` the
    algorithmic FLOP/s or B/s at the measured mean launch time (HIP events), `frac` = achieved / peak.
    The fused small-batch launches are latency chains over L2-resident intermediates: matrix roof only.
    `traffic` = measured HBM bytes per launch from the committed PMC summary of the same workload
    (null if none)."""
    avg_ms = float(np.mean(kern_ms))
    t = avg_ms * 1e-3
    fl_step = kernel_flops(kernel, Ne, Nn, S)
    kflops = fl_step / launches_per_step
    mpeak = MATH_PEAK[math]
    m_ach = kflops / t / 1e12
    by_step = None if (_FUSED[0] and kernel in FUSED_PARTS) else kernel_bytes(kernel, Ne, Nn, S, math)
    kbytes = by_step / launches_per_step if by_step else None
    b_ach = kbytes / t / 1e9 if kbytes else None
    traffic = load_pmc(config, kernel, math, workload)
    h_gbs = traffic / t / 1e9 if traffic else None
    hbm_bound = kbytes is not None and kbytes / (PEAK_HBM_GBS * 1e9) > kflops / (mpeak * 1e12)
    out = {"bound": "hbm" if hbm_bound else "mfma",
           "achieved": round(b_ach, 1) if hbm_bound else round(m_ach, 2),
           "peak": PEAK_HBM_GBS if hbm_bound else round(mpeak, 1),
           "unit": "GB/s" if hbm_bound else "TFLOP/s",
           "frac": round(b_ach / PEAK_HBM_GBS, 4) if hbm_bound else round(m_ach / mpeak, 4),
           "traffic": traffic, "kernel": kernel,
           "avg_launch_ms": round(avg_ms, 4), "launches": len(kern_ms), "launches_per_step": launches_per_step,
           "ms_per_step": round(avg_ms * launches_per_step, 4), "flop_per_launch": kflops,
           "alg_bytes_per_launch": round(kbytes) if kbytes else None,
           "intensity_flop_per_byte": round(kflops / kbytes, 1) if kbytes else None,
           "ridge_flop_per_byte": round(mpeak * 1e12 / (PEAK_HBM_GBS * 1e9), 1),
           "mfma_achieved_tflops": round(m_ach, 2), "mfma_frac": round(m_ach / mpeak, 4),
           "alg_hbm_gbs": round(b_ach, 1) if b_ach else None,
           "alg_hbm_frac": round(b_ach / PEAK_HBM_GBS, 4) if b_ach else None,
           "hbm_gbs": round(h_gbs, 1) if h_gbs else None,
           "hbm_frac": round(h_gbs / PEAK_HBM_GBS, 4) if h_gbs else None, "peak_note": PEAK_NOTE[math]}
    return out


def recorded_ms(ev, npairs):
    """Launch times of the event pairs the library recorded (pairs it did not record are skipped:
    a kernel runs fewer times than the slots reserved for it, or not at all in this math)."""
    out = []
    for i in range(npairs):
        try:
            out.append(ev.elapsed_ms(2 * i, 2 * i + 1))
        except RuntimeError:
            pass
    return out


def timed_steps(trainer, step_in, kid, n_micro, steps, slots):
    """`steps` training steps with HIP events around every launch of kernel `kid` (at most `slots`
    per micro-batch and step). Returns (launch ms list, launches per step, last step's out3)."""
    ev = HipEvents(2 * slots * n_micro * steps)
    per_step = 2 * slots * n_micro
    out3 = None
    for k in range(steps):
        evs = ev.ev[per_step * k: per_step * (k + 1)]
        if n_micro == 1:
            trainer.prof_kernel, trainer.prof_events = kid, evs
            out3 = trainer.step(*step_in)
        else:
            trainer.prof_kernel, trainer.prof_events = kid, None
            out3 = _micro_step(trainer, *step_in, evs, slots)
    trainer.prof_kernel, trainer.prof_events = 0, None
    torch.cuda.synchronize()
    ms = recorded_ms(ev, slots * n_micro * steps)
    ev.close()
    return ms, len(ms) // steps, out3


# ------------------------------------------------------------------------------ main
_JSON_OUT = None


def emit(out: dict) -> None:
    """The contract's ONE JSON line, on the process's original stdout (main() points fd 1 at stderr, so
    whatever a library prints — RCCL's version banner at communicator init — cannot precede it)."""
    f = _JSON_OUT if _JSON_OUT is not None else sys.stdout
    f.write(json.dumps(out) + "\n")
    f.flush()


def main():
    global _JSON_OUT
    sys.stdout.flush()
    _JSON_OUT = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=None, help="timed steps (default 10; 500 for replayed configs)")
    ap.add_argument("--warmup", type=int, default=None, help="untimed steps (default 3; 20 for replayed configs)")
    ap.add_argument("--config", type=int, default=0, choices=sorted(CONFIGS),
                    help="BASELINE.json config (1-5); 0 = the headline metric's configuration")
    ap.add_argument("--towers", type=int, default=None, help="towers per GPU (overrides the config)")
    ap.add_argument("--nodes", type=int, default=None)
    ap.add_argument("--mp-steps", type=int, default=None)
    ap.add_argument("--math", default=None, choices=["x6", "f32", "bf16"],
                    help="matrix-product arithmetic (spwgnn.h SPWGNN_MATH_*), overrides the config")
    ap.add_argument("--dropout", type=float, default=0.1)
    ap.add_argument("--roofline-kernel", default=None, choices=sorted(KERNELS))
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-f32-leg", action="store_true", help="skip the other-math reference measurements")
    ap.add_argument("--no-kernel-table", action="store_true", help="skip the per-kernel roofline table")
    ap.add_argument("--infer", action="store_true", help="alias of --config 5")
    ap.add_argument("--graph", action="store_true",
                    help="small-batch configs: replay each step as one captured hipGraph instead of issuing its "
                         "launches (the same sequence) eagerly — slower on the MI355X host (DESIGN.md §3x)")
    ap.add_argument("--buckets", type=int, default=1,
                    help="N>1 with --no-overlap: the flat gradient all-reduced as this many async pieces")
    ap.add_argument("--dist", action="store_true",
                    help="initialise the process group at one rank too (RCCL on the box's one GPU: the N>1 "
                         "step's collectives and overlap, over an identity all-reduce)")
    ap.add_argument("--no-overlap", action="store_true",
                    help="N>1: all-reduce the whole gradient after the backward instead of the early range "
                         "[rmp.1.kernel, end) during it (Trainer.reduce_split)")
    args = ap.parse_args()
    if args.infer:
        args.config = 5
    cfg = dict(CONFIGS[args.config])
    for k, a in (("towers", args.towers), ("nodes", args.nodes), ("S", args.mp_steps), ("math", args.math)):
        if a is not None:
            cfg[k] = a
    # a replayed step is ~0.4 ms: 10 of them are shorter than one host hiccup on a shared box, so
    # replayed configs time 500 (0.2 s) unless told otherwise
    if args.steps is None:
        args.steps = 500 if cfg.get("replay") else 10
    if args.warmup is None:
        args.warmup = 20 if cfg.get("replay") else 3

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # SPWGNN_DIST_BACKEND=gloo rehearses the N>1 path with every rank on the visible GPU(s)
    # (gloo all-reduces device tensors through the host); the driver's runs use nccl = RCCL
    backend = os.environ.get("SPWGNN_DIST_BACKEND", "nccl")
    if backend != "nccl":
        local = local % max(torch.cuda.device_count(), 1)
    if world > 1 or args.dist:
        if world == 1:   # --dist without a launcher: a one-rank group on this host
            for k, v in (("MASTER_ADDR", "127.0.0.1"), ("MASTER_PORT", "29547"), ("RANK", "0"), ("WORLD_SIZE", "1")):
                os.environ.setdefault(k, v)
        torch.cuda.set_device(local)
        if backend == "nccl":
            # RCCL on high-priority streams: the overlapped gradient piece runs beside the backward's
            # kernels instead of queueing behind them (Trainer.reduce_split)
            opts = dist.ProcessGroupNCCL.Options()
            opts.is_high_priority_stream = True
            dist.init_process_group("nccl", device_id=torch.device("cuda", local), pg_options=opts)
        else:
            dist.init_process_group(backend)
    device = torch.device("cuda", local)
    if cfg["mode"] == "infer":
        return run_infer(args, cfg, world, rank, device)
    return run_train(args, cfg, world, rank, device)


def run_train(args, cfg, world, rank, device):
    S, math = cfg["S"], cfg["math"]
    batches, targets, n_global = make_workload(cfg, rank, device, world)
    params = P.to_flat(P.glorot_uniform(0), device=device)
    dp = dist.is_available() and dist.is_initialized()   # a process group (N > 1, or --dist at one rank)
    if dp:
        dist.broadcast(params, 0)
    trainer = Trainer(params, mp_steps=S, dropout=args.dropout, seed=7, math=math, buckets=args.buckets,
                      overlap=not args.no_overlap)
    step_in = ((batches[0], targets[0]) if len(batches) == 1 else (batches, targets)) + (n_global,)
    n_micro = len(batches)
    for _ in range(args.warmup):
        trainer.step(*step_in)
    torch.cuda.synchronize()
    Ne = sum(b.n_edges for b in batches)
    Nn = sum(b.n_nodes for b in batches)
    B = sum(b.n_towers for b in batches)
    wl = workload_name(cfg, world, args.dropout)
    _FUSED[0] = fused_small(batches, math, S, args.dropout)

    # every timed kernel's per-step time, before the timed region (untimed steps), so the roofline
    # can name the DOMINANT kernel (largest ms per step) and time it inside the timed region
    table = {}
    if not args.no_kernel_table or not args.roofline_kernel:
        table = kernel_table(trainer, step_in, n_micro, S, Ne, Nn, math, args.config, wl)
    kname = args.roofline_kernel or dominant(table)
    kid = KERNELS[kname][0]
    if cfg.get("replay") and world == 1 and n_micro == 1 and not dp:
        return run_replay(args, cfg, trainer, rank, device, kname, table, wl)
    ev = HipEvents(2 * MAX_LAUNCHES * n_micro * args.steps)
    per = 2 * MAX_LAUNCHES * n_micro
    # N>1: the gradient all-reduce of every timed step between two events on the step's stream, so
    # the line separates the collective (RCCL over xGMI) from the compute
    ar_ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
             for _ in range(args.steps)] if dp else None
    # ... and, when the step overlaps (Trainer.reduce_split), the early piece's all-reduce on its side stream
    ar_early = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                for _ in range(args.steps)] if dp and trainer._split() else None
    if dp:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        # the library fills events in launch order: one slice of the array per step (and micro-batch)
        evs = ev.ev[per * k: per * (k + 1)]
        if ar_ev:
            trainer.ar_events = ar_ev[k]
        if ar_early:
            trainer.ar_early_events = ar_early[k]
        if n_micro == 1:
            trainer.prof_kernel, trainer.prof_events = kid, evs
            out3 = trainer.step(*step_in)
        else:
            trainer.prof_kernel, trainer.prof_events = kid, None
            out3 = _micro_step(trainer, *step_in, evs, MAX_LAUNCHES)
    torch.cuda.synchronize()
    if dp:
        dist.barrier()
    el = time.perf_counter() - t0
    trainer.prof_kernel, trainer.prof_events, trainer.ar_events, trainer.ar_early_events = 0, None, None, None
    allreduce = None
    if ar_ev:
        ar_ms = [a.elapsed_time(b) for a, b in ar_ev]
        ar_t = torch.tensor([float(np.mean(ar_ms))], dtype=torch.float64, device=device)
        dist.all_reduce(ar_t, op=dist.ReduceOp.MAX)
        nbytes = params.numel() * params.element_size()
        allreduce = {"allreduce_ms": round(float(ar_t.item()), 4), "bytes": nbytes, "buckets": trainer.buckets,
                     "backend": dist.get_backend(),
                     "note": "mean per step, max over ranks; HIP events on the step's stream from the end of the "
                             "backward to the gradients summed over ranks (the exposed all-reduce; includes "
                             "waiting for the slowest rank to arrive)"}
        if ar_early:
            lead = [a.elapsed_time(b) for (a, _), (b, _) in zip(ar_early, ar_ev)]
            dur = [a.elapsed_time(b) for a, b in ar_early]
            t2 = torch.tensor([float(np.min(lead)), float(np.mean(lead)), float(np.mean(dur))], dtype=torch.float64,
                              device=device)
            dist.all_reduce(t2, op=dist.ReduceOp.MIN)
            allreduce["overlap"] = {
                "early_range_floats": int(params.numel() - trainer._early_lo),
                "early_start_before_backward_end_ms": {"min": round(float(t2[0]), 4), "mean": round(float(t2[1]), 4)},
                "early_piece_ms": round(float(t2[2]), 4),
                "note": "Trainer.reduce_split: the gradients of [rmp.1.kernel, end) all-reduced on a side stream "
                        "from the backward's early event (spwgnn_run.grads_early_event); lead = its start to the end "
                        "of the backward (> 0: it ran while dA, the encoder backward and the encoder-side "
                        "gradients did), min over ranks"}
    el_t = torch.tensor([el], dtype=torch.float64, device=device)
    if dp:
        dist.all_reduce(el_t, op=dist.ReduceOp.MAX)
    el = float(el_t.item())
    kern_ms = recorded_ms(ev, MAX_LAUNCHES * n_micro * args.steps)
    ev.close()
    loss = float(out3[0].item())     # node-weighted mean BCE over this rank's micro-batches

    roof = roofline(kname, kern_ms, len(kern_ms) // args.steps, Ne, Nn, S, math, args.config, wl)
    roof["selected"] = "--roofline-kernel" if args.roofline_kernel else \
        "dominant: largest ms per step in this run's kernel table (measured before the timed region)"
    metric = METRIC if args.config == 0 else f"towers/sec fwd+bwd, BASELINE config {args.config}"
    out = {
        "metric": metric,
        "value": round(cfg["towers"] * world * args.steps / el, 1),   # the whole global batch per step
        "unit": "towers/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(el / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "bf16" if math == "bf16" else "f32",
        "math": MATH_DESC[math],
        "data": "synthetic (Jenga-geometry towers, random labels, glorot weights)",
        "config": {"workload": wl, "baseline_config": args.config, "towers_per_gpu": B, "global_batch": cfg["towers"] * world,
                   "n_global_nodes": n_global, "shard_plan": "shard.plan_shards (cost-balanced contiguous ranges)",
                   "nodes_per_tower": list(cfg["nodes"]) if isinstance(cfg["nodes"], tuple) else cfg["nodes"],
                   "nodes_per_gpu": Nn, "edges_per_gpu": Ne, "mp_steps": S, "math": math,
                   "parallelism": f"dp{world}" + (" (one-rank process group)" if dp and world == 1 else "")},
        "step_tflops": round(step_flops(Ne, Nn, S) * world * args.steps / el / 1e12, 2),
        "loss": round(loss, 5),
        "roofline": roof,
        "cpu_baseline": None,
    }
    if allreduce:
        out["allreduce_ms"] = allreduce["allreduce_ms"]
        out["allreduce"] = allreduce
    if world == 1 and args.config == 0 and math == "x6" and not args.no_f32_leg:
        # the same step in the other SPWGNN_MATH_* modes, for reference: f32 MFMA (fp32-class like
        # x6) and bf16 (operands rounded to bf16, one product — BASELINE configs 3-4's arithmetic)
        for m in ("f32", "bf16"):
            trm = Trainer(params.clone(), mp_steps=S, dropout=args.dropout, seed=7, math=m)
            for _ in range(2):
                trm.step(*step_in)
            torch.cuda.synchronize()
            km = max(3, args.steps // 2)
            t1 = time.perf_counter()
            for _ in range(km):
                trm.step(*step_in)
            torch.cuda.synchronize()
            em = time.perf_counter() - t1
            out[f"{m}_math"] = {"value": round(B * km / em, 1), "ms_per_step": round(em / km * 1e3, 3), "steps": km}
            del trm
            torch.cuda.empty_cache()
    out["hbm"] = step_hbm(args.config, out["ms_per_step"], math, wl)
    if table and not args.no_kernel_table:
        out["kernels"] = table
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(cfg, args.cpu_seconds)
    if rank == 0:
        emit(out)
    if dp:
        dist.destroy_process_group()


def run_replay(args, cfg, trainer, rank, device, kname, table, wl):
    """A launch-bound config (config 1: the reference's own 32-tower batch) timed as it should run: the
    replayable step of spwgnn_amd/replay.py — static device buffers refilled from a pinned staging
    slot by the step's first launch, the dropout key and Adam step as device words — issued eagerly
    (the host keeps ahead of the GPU; `--graph` replays the same step as one captured hipGraph,
    ≈ 4 µs slower per step on the MI355X host). The batch is planned with every
    relation slot (N(N−1) per tower); the kernel table and roofline come from eager steps of the same
    trainer."""
    from spwgnn_amd.replay import ReplayStep
    S, math = cfg["S"], cfg["math"]
    plans, tg_np, n_global = make_workload(cfg, rank, device, 1, plans=True)
    plan, tgt = plans[0], tg_np[0]
    rs = ReplayStep(plan, device, trainer.replay_body(plan.n_nodes, n_global), graph=args.graph)
    for _ in range(args.warmup + 1):             # the first call runs eagerly and captures
        trainer.replay_step(rs, plan, tgt)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        trainer.replay_step(rs, plan, tgt)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    loss = float(rs.bce.out3[0].item())
    Ne, Nn = len(plan.src), plan.n_nodes
    k = table.get(kname)
    roof = None
    if k:
        roof = roofline(kname, [k["avg_launch_ms"]], k["launches_per_step"], Ne, Nn, S, math, args.config, wl)
        roof["selected"] = "dominant kernel of this run's kernel table (eager steps of the same batch)"
    out = {
        "metric": f"towers/sec fwd+bwd, BASELINE config {args.config}", "value": round(cfg["towers"] * args.steps / el, 1),
        "unit": "towers/s", "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(el / args.steps * 1e3, 4), "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "bf16" if math == "bf16" else "f32", "math": MATH_DESC[math],
        "data": "synthetic (Jenga-geometry towers, random labels, glorot weights)",
        "config": {"workload": wl, "step_mode": ("each step one replayed hipGraph (batch arrays copied in by its first launch)"
                                                  if args.graph else "each step's launches issued eagerly from static buffers "
                                                  "(batch arrays copied in by its first launch; --graph: the same step replayed)"),
                   "baseline_config": args.config, "towers_per_gpu": cfg["towers"], "global_batch": cfg["towers"],
                   "nodes_per_tower": cfg["nodes"], "nodes_per_gpu": Nn, "edges_per_gpu": Ne, "mp_steps": S,
                   "math": math, "parallelism": "dp1", "replays": rs.replays, "eblocks_planned": plan.n_eblocks},
        "step_tflops": round(step_flops(Ne, Nn, S) * args.steps / el / 1e12, 4),
        "loss": round(loss, 5), "roofline": roof, "kernels": table, "cpu_baseline": None,
    }
    out["hbm"] = step_hbm(args.config, out["ms_per_step"], math, wl)
    if rank == 0 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(cfg, args.cpu_seconds)
    emit(out)


# kernel families: one SPWGNN_K_* id over several weight-gradient shapes. Batched (the default:
# k_wgrad_ws_batch, one launch per backward) the family IS one kernel and can be named dominant;
# unbatched (SPWGNN_WS_UNBATCHED, one launch per shape) it is listed but never named — a roofline
# belongs to one kernel.
FAMILIES = ("wgrad_ws",)


def dominant(table) -> str:
    """The single kernel with the largest time per step in this run's kernel table."""
    single = {k: v for k, v in table.items() if k not in FAMILIES or v.get("batched")}
    return max(single, key=lambda k: single[k]["ms_per_step"]) if single else "edge_fwd"


def kernel_table(trainer, step_in, n_micro, S, Ne, Nn, math, config, wl, steps=2, names=None):
    """Every timed kernel's roofline in the same run: `steps` extra (untimed) training steps per kernel
    with HIP events around each of its launches (the library's prof hook takes one kernel id per call).
    Per kernel: launches and ms per step, mean launch ms, achieved TFLOP/s, frac of the math's matrix
    peak, measured HBM bytes per launch from the committed PMC summary of this workload."""
    table = {}
    for name in names or KERNELS:
        kid = KERNELS[name][0]
        ms, per_step, _ = timed_steps(trainer, step_in, kid, n_micro, steps, MAX_LAUNCHES)
        if not ms:
            continue   # kernel not launched by this configuration / math
        r = roofline(name, ms, per_step, Ne, Nn, S, math, config, wl)
        table[name] = {"launches_per_step": per_step, "avg_launch_ms": r["avg_launch_ms"],
                       "ms_per_step": r["ms_per_step"], "tflops": r["mfma_achieved_tflops"], "frac": r["mfma_frac"],
                       "bound": r["bound"], "roof_frac": r["frac"], "alg_hbm_frac": r["alg_hbm_frac"],
                       "traffic": r["traffic"], "hbm_gbs": r["hbm_gbs"]}
        if _FUSED[0] and name in FUSED_PARTS:
            table[name]["fused"] = "+".join(FUSED_PARTS[name])
        if name in FAMILIES:
            table[name]["batched"] = bool(per_step <= n_micro)
            table[name]["family"] = ("one launch per backward batching every weight-gradient shape (k_wgrad_ws_batch)"
                                     if per_step <= n_micro else
                                     "several kernels of different shapes under one id; frac over the family")
    return table


def _micro_step(trainer, batches, targets, n_global, evs, per_mb):
    """Trainer.step over micro-batches with the timed kernel's events handed to each micro-batch's
    launches (the library records at most prof_count pairs per call)."""
    orig = trainer.run_config

    def rc(micro=0):
        r = orig(micro)
        r.prof_kernel = trainer_kid[0]
        r.prof_events = evs[2 * per_mb * micro: 2 * per_mb * (micro + 1)]
        return r
    trainer_kid = [trainer.prof_kernel]
    trainer.run_config = rc
    try:
        return trainer.step(batches, targets, n_global)
    finally:
        trainer.run_config = orig


INFER_METRIC = "towers/sec fwd (inference), 32-block towers, 10 MP steps, hipGraph-captured forward"


def run_infer(args, cfg, world, rank, device):
    """Config 5: the forward of a whole batch captured once into a hipGraph (torch.cuda.CUDAGraph
    over the library's launches on the capture stream) and replayed; weak scaling, replicas."""
    from spwgnn_amd import engine as E
    B, N, S, math = cfg["towers"], cfg["nodes"], cfg["S"], cfg["math"]
    raw = D.synthetic_towers_fast(B, N, seed=5000 + rank)
    batch = TowerBatch.fully_connected((raw / D.RELATION_THRESHOLD).astype(np.float32), device=device)
    params = P.to_flat(P.glorot_uniform(0), device=device)
    run = E.RunConfig(S, training=False, math=math)
    ws = E.Workspace(device)
    z = torch.empty(batch.n_nodes, dtype=torch.float32, device=device)
    side = torch.cuda.Stream(device)
    side.wait_stream(torch.cuda.current_stream(device))
    with torch.cuda.stream(side):
        E.forward(params, batch, run, ws, logits=z)      # sizes the workspace before capture
    torch.cuda.current_stream(device).wait_stream(side)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        E.forward(params, batch, run, ws, logits=z)
    for _ in range(args.warmup):
        graph.replay()
    torch.cuda.synchronize()
    # every forward kernel timed with HIP events on un-captured passes (same stream, same launches);
    # the roofline names the dominant one (largest ms per forward)
    Ne, Nn = batch.n_edges, batch.n_nodes
    wl = workload_name(cfg, world, 0.0)
    table, times = {}, {}
    for name in INFER_KERNELS:
        ev = HipEvents(2 * MAX_LAUNCHES * 3)
        for k in range(3):
            evs = ev.ev[2 * MAX_LAUNCHES * k: 2 * MAX_LAUNCHES * (k + 1)]
            prun = E.RunConfig(S, training=False, math=math, prof_kernel=KERNELS[name][0], prof_events=evs)
            E.forward(params, batch, prun, ws, logits=z)
        torch.cuda.synchronize()
        ms = recorded_ms(ev, MAX_LAUNCHES * 3)
        ev.close()
        if not ms:
            continue
        r = roofline(name, ms, len(ms) // 3, Ne, Nn, S, math, 5, wl)
        times[name] = ms
        table[name] = {"launches_per_step": len(ms) // 3, "avg_launch_ms": r["avg_launch_ms"],
                       "ms_per_step": r["ms_per_step"], "tflops": r["mfma_achieved_tflops"], "frac": r["mfma_frac"],
                       "bound": r["bound"], "roof_frac": r["frac"], "alg_hbm_frac": r["alg_hbm_frac"],
                       "traffic": r["traffic"], "hbm_gbs": r["hbm_gbs"]}
    kname = args.roofline_kernel or dominant(table)
    if kname not in times:
        raise SystemExit(f"kernel {kname} is not launched by the inference forward")
    kern_ms = times[kname]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        graph.replay()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    el_t = torch.tensor([el], dtype=torch.float64, device=device)
    if world > 1:
        dist.all_reduce(el_t, op=dist.ReduceOp.MAX)
    el = float(el_t.item())
    out = {
        "metric": INFER_METRIC, "value": round(world * B * args.steps / el, 1), "unit": "towers/s",
        "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(el / args.steps * 1e3, 3), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "bf16" if math == "bf16" else "f32", "math": MATH_DESC[math],
        "data": "synthetic (Jenga-geometry towers, glorot weights)",
        "config": {"workload": wl, "baseline_config": 5, "towers_per_gpu": B, "global_batch": cfg["towers"] * world,
                   "nodes_per_tower": N, "mp_steps": S, "math": math, "parallelism": f"replicas{world}"},
        "step_tflops": round(fwd_flops(Ne, Nn, S) * world * args.steps / el / 1e12, 2),
        "roofline": dict(roofline(kname, kern_ms, len(kern_ms) // 3, Ne, Nn, S, math, 5, wl),
                         selected="--roofline-kernel" if args.roofline_kernel else
                         "dominant: largest ms per forward in this run's kernel table"),
        "kernels": table,
        "cpu_baseline": None,
    }
    out["hbm"] = step_hbm(5, out["ms_per_step"], math, wl)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(cfg, args.cpu_seconds)
    if rank == 0:
        emit(out)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
