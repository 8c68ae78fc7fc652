#!/usr/bin/env python3
"""Benchmark: towers/s of one full training step (forward + BCE + backward [+ RCCL all-reduce] +
Adam) on synthetic 6-block Jenga towers, 65,536 towers per GPU, 5 propagation steps, fp32.

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
from spwgnn_amd.batch import TowerBatch  # noqa: E402
from spwgnn_amd.trainer import Trainer  # noqa: E402

METRIC = "towers/sec fwd+bwd, 6-block batch=65k, 1/2/4/8 MI355X; achieved HBM GB/s"
PEAK_FP32_TFLOPS = 157.3    # MI355X_MICROARCH.md: fp32 MFMA (= vector) peak
PEAK_BF16_TFLOPS = 2500.0   # MI355X_MICROARCH.md: dense bf16 MFMA peak
PEAK_HBM_GBS = 8000.0
# x6 math runs each fp32 product as 6 bf16 MFMA products: its fp32-equivalent matrix peak
PEAK_X6_TFLOPS = PEAK_BF16_TFLOPS / 6

# algorithmic FLOPs per launch of each timed kernel, as f(real edges, nodes, S)
KERNELS = {
    "edge_fwd": (_lib.K_EDGE_FWD, lambda Ne, Nn, S: 2.0 * 150 * 150 * Ne),
    "edge_bwd": (_lib.K_EDGE_BWD, lambda Ne, Nn, S: 2.0 * 150 * 150 * Ne),
    "wgrad_w2": (_lib.K_WGRAD_W2, lambda Ne, Nn, S: 2.0 * 151 * 150 * Ne * S),
    "enc_edge": (_lib.K_ENC_EDGE, lambda Ne, Nn, S: 2.0 * (2 * 150 + 4 * 150 * 150) * Ne),
    "enc_edge_bwd": (_lib.K_ENC_EDGE_BWD, lambda Ne, Nn, S: 2.0 * 4 * 150 * 150 * Ne),
}
LAUNCHES_PER_STEP = {"edge_fwd": "S", "edge_bwd": "S", "wgrad_w2": 1, "enc_edge": 1, "enc_edge_bwd": 1}


def step_flops(Ne: int, Nn: int, S: int) -> float:
    """Algorithmic FLOPs of one fwd+bwd training step in the form the kernels compute."""
    fwd = Ne * (2 * 150 + 4 * 150 * 150) + Nn * (2 * 100 + 100 * 100) \
        + S * (Ne * 150 * 150 + Nn * (151 * 100 + 300 * 100 + 100 * 101 + 2 * 100 * 150)) - Nn * 2 * 100 * 150
    bwd_edge = Ne * (4 * 150 * 150 + 4 * 151 * 150 + 3 * 100) + S * Ne * (150 * 150 + 151 * 150)
    bwd_node = Nn * (100 * 100 + 101 * 100 + 3 * 100) + S * Nn * (
        2 * 150 * 100 + 101 * 100 + 300 * 100 + 150 * 100     # activation grads
        + 2 * 100 * 150 + 151 * 100 + 301 * 100 + 101 * 101)  # weight grads
    return 2.0 * (fwd + bwd_edge + bwd_node)


class HipEvents:
    def __init__(self, n):
        self.hip = C.CDLL("libamdhip64.so")
        self.ev = []
        for _ in range(n):
            e = C.c_void_p()
            if self.hip.hipEventCreate(C.byref(e)) != 0:
                raise RuntimeError("hipEventCreate failed")
            self.ev.append(e.value)

    def elapsed_ms(self, a, b) -> float:
        ms = C.c_float()
        self.hip.hipEventSynchronize(C.c_void_p(self.ev[b]))
        st = self.hip.hipEventElapsedTime(C.byref(ms), C.c_void_p(self.ev[a]), C.c_void_p(self.ev[b]))
        if st != 0:
            raise RuntimeError(f"hipEventElapsedTime failed ({st})")
        return ms.value

    def close(self):
        for e in self.ev:
            self.hip.hipEventDestroy(C.c_void_p(e))


def cpu_baseline_pair(n_objects: int, S: int, seconds: float):
    """The oracle at up to 16 host threads (the reported baseline) and at 1 thread."""
    many = cpu_baseline(n_objects, S, seconds)
    one = cpu_baseline(n_objects, S, max(3.0, seconds / 3), threads=1)
    many["value_1thread"] = one["value"]
    many["sample"] += f"; 1 thread: {one['value']:.1f} towers/s ({one['sample'].split(', ')[2]})"
    return many


def cpu_baseline(n_objects: int, S: int, seconds: float, threads=None):
    """The oracle (torch-CPU restatement of Networks.py, literal dense one-hot form, fp32 like
    Keras floatx) timed fwd+bwd on a bounded sample on this host's cores."""
    from oracle import model as O
    threads = max(1, min(16, len(os.sched_getaffinity(0)))) if threads is None else threads
    torch.set_num_threads(threads)
    B = 256
    obj, Rs, Rr, prop, tgt = D.synthetic_batch(B, n_objects, seed=123, fully_connected=True)
    p = O.to_torch(O.glorot_uniform_params(0), dtype=torch.float32, requires_grad=True)
    ts = [torch.tensor(a, dtype=torch.float32) for a in (obj, Rs, Rr, prop)]
    t = torch.tensor(tgt, dtype=torch.float32)

    def one():
        for v in p.values():
            v.grad = None
        z = O.forward_dense(p, *ts, S)
        O.keras_bce_from_logits(z, t).backward()

    one()
    n, t0 = 0, time.perf_counter()
    while True:
        one()
        n += 1
        el = time.perf_counter() - t0
        if (el > seconds and n >= 3) or n >= 200:
            break
    return {"value": B * n / el, "unit": "towers/s", "cores": threads, "kind": "port",
            "sample": f"oracle.forward_dense fp32 fwd+bwd, {B} towers x {n} iters, N={n_objects}, S={S}, "
                      f"{el:.1f}s, torch CPU threads={threads}"}


# device kernel whose PMC summary (profiles/pmc_summary.json, tools/pmcsum.py) holds the HBM
# bytes of a bench kernel
PMC_NAMES = {
    "f32": {"edge_fwd": "k_edge_fwd<true>", "edge_bwd": "k_edge_bwd<true, true>", "enc_edge": "k_enc_edge<true>",
            "enc_edge_bwd": "k_enc_edge_bwd", "wgrad_w2": "k_wgrad_t<4, 2, 160, 160>"},
    "x6": {"edge_fwd": "k_edge_fwd_x6<true, 0, 3>", "edge_bwd": "k_edge_bwd_x6<true, 0, 3>",
           "enc_edge": "k_enc_edge_x6<true, 2, 3>", "enc_edge_bwd": "k_enc_edge_bwd_x6<2, 3>",
           "wgrad_w2": "k_w2grad_ws<0, 3>"},
}


PMC_WORKLOAD = (65536, 6, 5)   # (towers per GPU, nodes, MP steps) of profiles/pmc_summary.json


def load_pmc(kernel: str, math: str = "x6"):
    """HBM bytes per launch (FETCH_SIZE x2 gfx950 correction + WRITE_SIZE) from the committed PMC
    summary, or None when absent."""
    path = os.path.join(ROOT, "profiles", "pmc_summary.json")
    name = PMC_NAMES.get(math, {}).get(kernel)
    if name is None or not os.path.exists(path):
        return None
    try:
        with open(path) as f:
            d = json.load(f).get(name, {})
        if "hbm_read_bytes" not in d or "hbm_write_bytes" not in d:
            return None
        return float(d["hbm_read_bytes"] + d["hbm_write_bytes"])
    except Exception:
        return None


def step_hbm(ms_per_step: float):
    """Whole-step HBM bytes from the committed PMC summary (one entry per kernel: mean bytes per
    dispatch × dispatches; the summary's run covers as many steps as k_adam dispatches)."""
    path = os.path.join(ROOT, "profiles", "pmc_summary.json")
    if not os.path.exists(path):
        return None
    try:
        with open(path) as f:
            d = json.load(f)
        steps = d.get("k_adam", {}).get("dispatches", 0)
        if not steps:
            return None
        tot = sum(v.get("hbm_read_bytes", 0.0) * v["dispatches"] + v.get("hbm_write_bytes", 0.0) * v["dispatches"]
                  for v in d.values() if "dispatches" in v)
        per = tot / steps
        gbs = per / (ms_per_step * 1e-3) / 1e9
        return {"bytes_per_step": round(per), "achieved_gbs": round(gbs, 1), "peak_gbs": PEAK_HBM_GBS,
                "frac": round(gbs / PEAK_HBM_GBS, 4),
                "source": "profiles/pmc_summary.json (rocprofv3 FETCH_SIZE x2 + WRITE_SIZE per kernel)"}
    except Exception:
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--towers", type=int, default=65536, help="towers per GPU")
    ap.add_argument("--nodes", type=int, default=6)
    ap.add_argument("--mp-steps", type=int, default=5)
    ap.add_argument("--dropout", type=float, default=0.1)
    ap.add_argument("--roofline-kernel", default="edge_bwd", choices=sorted(KERNELS))
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-f32-leg", action="store_true", help="skip the f32-math reference measurement")
    ap.add_argument("--math", default="x6", choices=["x6", "f32", "bf16"],
                    help="matrix-product arithmetic (spwgnn.h SPWGNN_MATH_*)")
    ap.add_argument("--infer", action="store_true",
                    help="BASELINE config 5: forward-only inference replayed from a hipGraph "
                         "(defaults: 32-block towers, S=10, 8192 towers/GPU)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # SPWGNN_DIST_BACKEND=gloo rehearses the N>1 path with every rank on the visible GPU(s)
    # (gloo all-reduces device tensors through the host); the driver's runs use nccl = RCCL
    backend = os.environ.get("SPWGNN_DIST_BACKEND", "nccl")
    if backend != "nccl":
        local = local % max(torch.cuda.device_count(), 1)
    if world > 1:
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    device = torch.device("cuda", local)

    if args.infer:
        return run_infer(args, world, rank, device)
    B, N, S = args.towers, args.nodes, args.mp_steps
    raw = D.synthetic_towers(B, N, seed=1000 + rank)
    objects = (raw / D.RELATION_THRESHOLD).astype(np.float32)
    batch = TowerBatch.fully_connected(objects, device=device)
    rng = np.random.default_rng(rank)
    target = torch.tensor(rng.integers(0, 2, size=B * N).astype(np.float32), device=device)
    params = P.to_flat(P.glorot_uniform(0), device=device)
    if world > 1:
        dist.broadcast(params, 0)
    trainer = Trainer(params, mp_steps=S, dropout=args.dropout, seed=7, math=args.math)

    for _ in range(args.warmup):
        trainer.step(batch, target)
    torch.cuda.synchronize()

    kid, flops_fn = KERNELS[args.roofline_kernel]
    per = LAUNCHES_PER_STEP[args.roofline_kernel]
    nl = (S if per == "S" else per) * args.steps
    ev = HipEvents(2 * nl)
    trainer.prof_kernel = kid
    trainer.prof_events = ev.ev
    # the library fills events in launch order; re-offset the array every step
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    per_step = nl // args.steps
    for k in range(args.steps):
        trainer.prof_events = ev.ev[2 * per_step * k: 2 * per_step * (k + 1)]
        out3 = trainer.step(batch, target)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    el_t = torch.tensor([el], dtype=torch.float64, device=device)
    if world > 1:
        dist.all_reduce(el_t, op=dist.ReduceOp.MAX)
    el = float(el_t.item())
    kern_ms = [ev.elapsed_ms(2 * i, 2 * i + 1) for i in range(nl)]
    ev.close()
    loss = float(out3[0].item())

    Ne, Nn = batch.n_edges, batch.n_nodes
    avg_ms = float(np.mean(kern_ms))
    kflops = flops_fn(Ne, Nn, S)
    achieved = kflops / (avg_ms * 1e-3) / 1e12
    value = world * B * args.steps / el
    total_flops = step_flops(Ne, Nn, S)
    # roofline of the timed kernel: its algorithmic fp32 FLOPs against the matrix peak of the math
    # it runs in (x6: bf16 peak / 6); its PMC HBM bytes per launch are reported as `traffic`
    mpeak = {"x6": PEAK_X6_TFLOPS, "f32": PEAK_FP32_TFLOPS, "bf16": PEAK_BF16_TFLOPS}[args.math]
    # the committed PMC summary was collected at the default workload (tools/round_artifacts.sh):
    # its bytes are only quoted for that shape
    pmc_shape = (B, N, S) == PMC_WORKLOAD
    traffic = load_pmc(args.roofline_kernel, args.math) if pmc_shape else None
    m_frac = achieved / mpeak
    h_gbs = traffic / (avg_ms * 1e-3) / 1e9 if traffic else None
    h_frac = h_gbs / PEAK_HBM_GBS if h_gbs else None
    # every timed kernel is fused GEMM work far above the ridge point (≫ 100 algorithmic
    # FLOP per compulsory HBM byte), so its roofline is the matrix pipe: achieved = algorithmic FLOPs
    # per launch ÷ mean launch time. The PMC bytes are the measured traffic beside it (hbm_gbs is
    # that traffic's rate, not an algorithmic figure).
    roof = {"bound": "mfma", "achieved": round(achieved, 2), "peak": round(mpeak, 1), "unit": "TFLOP/s",
            "frac": round(m_frac, 4)}
    roof.update({"kernel": args.roofline_kernel, "traffic": traffic, "avg_launch_ms": round(avg_ms, 4),
                 "launches": nl, "flop_per_launch": kflops, "mfma_tflops": round(achieved, 2),
                 "mfma_peak": round(mpeak, 1), "mfma_frac": round(m_frac, 4),
                 "hbm_gbs": round(h_gbs, 1) if h_gbs else None, "hbm_frac": round(h_frac, 4) if h_frac else None,
                 "peak_note": {"x6": "x6: fp32 products as 6 bf16 MFMA products, peak = 2.5 PF bf16 / 6",
                               "f32": "f32 MFMA peak", "bf16": "bf16 MFMA dense peak"}[args.math]})
    out = {
        "metric": METRIC,
        "value": round(value, 1),
        "unit": "towers/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(el / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "bf16" if args.math == "bf16" else "f32",
        "math": {"x6": "x6: each fp32 matrix product as 6 bf16 MFMA products of 3-way split operands, fp32 "
                       "accumulation (DESIGN.md §3b)", "f32": "f32 MFMA",
                 "bf16": "bf16: operands rounded to bf16, one bf16 MFMA product, fp32 accumulation"}[args.math],
        "data": "synthetic (Jenga-geometry towers, random labels, glorot weights)",
        "config": {"workload": f"train step fwd+BCE+bwd+{'allreduce+' if world > 1 else ''}Adam, "
                               f"{N}-block towers fully connected (E={N*(N-1)}), {B} towers/GPU, "
                               f"{S} MP steps, dropout {args.dropout}",
                   "towers_per_gpu": B, "global_batch": B * world, "nodes_per_tower": N, "mp_steps": S,
                   "parallelism": f"dp{world}"},
        "step_tflops": round(total_flops * world * args.steps / el / 1e12, 2),
        "loss": round(loss, 5),
        "roofline": roof,
        "cpu_baseline": None,
    }
    if world == 1 and args.math == "x6" and not args.no_f32_leg:
        # the same step in the other SPWGNN_MATH_* modes, for reference: f32 MFMA (fp32-class like
        # x6) and bf16 (operands rounded to bf16, one product — BASELINE configs 3-4's arithmetic)
        for m in ("f32", "bf16"):
            trm = Trainer(params.clone(), mp_steps=S, dropout=args.dropout, seed=7, math=m)
            for _ in range(2):
                trm.step(batch, target)
            torch.cuda.synchronize()
            km = max(3, args.steps // 2)
            t1 = time.perf_counter()
            for _ in range(km):
                trm.step(batch, target)
            torch.cuda.synchronize()
            em = time.perf_counter() - t1
            out[f"{m}_math"] = {"value": round(B * km / em, 1), "ms_per_step": round(em / km * 1e3, 3), "steps": km}
            del trm
            torch.cuda.empty_cache()
    out["hbm"] = step_hbm(out["ms_per_step"]) if pmc_shape else None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline_pair(N, S, args.cpu_seconds)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


INFER_METRIC = "towers/sec fwd (inference), 32-block towers, 10 MP steps, hipGraph-captured forward"


def run_infer(args, world, rank, device):
    """Config 5: the forward of a whole batch captured once into a hipGraph (torch.cuda.CUDAGraph
    over the library's launches on the capture stream) and replayed; weak scaling, replicas."""
    from spwgnn_amd import engine as E
    B = args.towers if args.towers != 65536 else 8192
    N = args.nodes if args.nodes != 6 else 32
    S = args.mp_steps if args.mp_steps != 5 else 10
    raw = D.synthetic_towers(B, N, seed=5000 + rank)
    batch = TowerBatch.fully_connected((raw / D.RELATION_THRESHOLD).astype(np.float32), device=device)
    params = P.to_flat(P.glorot_uniform(0), device=device)
    run = E.RunConfig(S, training=False)
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
    # dominant kernel timed with HIP events on an un-captured pass (same stream, same launches)
    kid, flops_fn = _lib.K_EDGE_FWD, KERNELS["edge_fwd"][1]
    ev = HipEvents(2 * S)
    prun = E.RunConfig(S, training=False, prof_kernel=kid, prof_events=ev.ev)
    E.forward(params, batch, prun, ws, logits=z)
    torch.cuda.synchronize()
    kern_ms = [ev.elapsed_ms(2 * i, 2 * i + 1) for i in range(S)]
    ev.close()
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
    Ne, Nn = batch.n_edges, batch.n_nodes
    avg_ms = float(np.mean(kern_ms))
    kflops = flops_fn(Ne, Nn, S)
    achieved = kflops / (avg_ms * 1e-3) / 1e12
    # forward FLOPs as the kernels compute them (rmp layer 3 behind the receiver sum)
    fwd_flops = 2.0 * (Ne * (2 * 150 + 4 * 150 * 150) + Nn * (2 * 100 + 100 * 100)
                       + S * (Ne * 150 * 150 + Nn * (151 * 100 + 300 * 100 + 100 * 101 + 2 * 100 * 150))
                       - Nn * 2 * 100 * 150)
    out = {
        "metric": INFER_METRIC, "value": round(world * B * args.steps / el, 1), "unit": "towers/s",
        "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(el / args.steps * 1e3, 3), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "fp32", "data": "synthetic (Jenga-geometry towers, glorot weights)",
        "config": {"workload": f"forward, {N}-block towers fully connected (E={N * (N - 1)}), {B} towers/GPU, "
                               f"{S} MP steps, hipGraph replay", "towers_per_gpu": B, "global_batch": B * world,
                   "nodes_per_tower": N, "mp_steps": S, "parallelism": f"replicas{world}"},
        "step_tflops": round(fwd_flops * world * args.steps / el / 1e12, 2),
        "roofline": {"kernel": "edge_fwd", "bound": "mfma", "achieved": round(achieved, 2),
                     "peak": PEAK_FP32_TFLOPS, "unit": "TFLOP/s", "frac": round(achieved / PEAK_FP32_TFLOPS, 4),
                     "avg_launch_ms": round(avg_ms, 4), "launches": S, "flop_per_launch": kflops, "traffic": None},
        "cpu_baseline": None,
    }
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
