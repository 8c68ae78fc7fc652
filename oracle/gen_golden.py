"""Generate the committed golden vectors under tests/golden/ from the fp64 oracle.

PARITY UNPINNED: the reference (Keras 2.x / TF 1.x) cannot run here and ships no fixtures, so
these vectors come from this repo's own oracle (oracle/model.py, a line-by-line restatement of
src/Networks.py + src/Blocks.py). They pin the oracle and the engine against regressions and give
the GPU tests fixtures that need no oracle at run time.

Run:  python -m oracle.gen_golden
"""
from __future__ import annotations

import os

import numpy as np

from . import model as O
from . import dropout as DR

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(os.path.dirname(HERE), "tests", "golden")


def _towers(B, N, seed):
    # inline copy of the synthetic geometry (JengaBuilder.py:137-192) would duplicate product code;
    # golden inputs are plain seeded boxes in the same pixel ranges instead.
    rng = np.random.default_rng(seed)
    raw = np.zeros((B, N, 3))
    for b in range(B):
        for i in range(N):
            layer = i // 2
            raw[b, i] = [rng.uniform(400, 1100), 110 + 80 * layer + rng.uniform(-2, 2), rng.integers(50, 301)]
    return raw


def main():
    os.makedirs(OUT, exist_ok=True)
    params = O.random_params(seed=2024)
    np.savez_compressed(os.path.join(OUT, "golden_params.npz"), **params)
    for N, B, S, fully in [(3, 4, 5, True), (5, 4, 5, False), (6, 4, 5, False), (6, 3, 1, True),
                           (9, 2, 5, False), (12, 2, 3, True)]:
        raw = _towers(B, N, seed=100 + N)
        Rs, Rr = O.relation_matrices(raw, None if fully else O.RELATION_THRESHOLD)
        objects = (raw / O.RELATION_THRESHOLD).astype(np.float32)
        rng = np.random.default_rng(N)
        prop = (rng.normal(0, 0.2, size=(B, N, 100)) if N == 5 else np.zeros((B, N, 100))).astype(np.float32)
        target = rng.integers(0, 2, size=(B, N)).astype(np.float32)
        loss, logits, grads = O.loss_and_grads(params, objects, Rs, Rr, prop, target, S)
        rec = dict(objects=objects, Rs=Rs.astype(np.float32), Rr=Rr.astype(np.float32), prop=prop, target=target,
                   mp_steps=np.int32(S), logits=logits, loss=np.float64(loss))
        full = (N == 6 and S == 5)
        for k, g in grads.items():
            if full:
                rec["grad/" + k] = g.astype(np.float64)
            else:
                idx = np.random.default_rng(7).choice(g.size, size=min(64, g.size), replace=False)
                rec["gidx/" + k] = idx.astype(np.int64)
                rec["gval/" + k] = g.reshape(-1)[idx].astype(np.float64)
                rec["gsum/" + k] = np.float64(g.sum())
        tag = f"N{N}_B{B}_S{S}_{'full' if fully else 'thr'}"
        np.savez_compressed(os.path.join(OUT, f"golden_{tag}.npz"), **rec)
        print("wrote", tag, "loss", loss)
    # dropout fixture: masks from the engine's key, oracle run with them (B=2, N=6)
    B, N, S, seed, rate = 2, 6, 5, 123456789, 0.1
    raw = _towers(B, N, seed=77)
    Rs, Rr = O.relation_matrices(raw, None)
    objects = (raw / O.RELATION_THRESHOLD).astype(np.float32)
    prop = np.zeros((B, N, 100), np.float32)
    target = np.random.default_rng(3).integers(0, 2, size=(B, N)).astype(np.float32)
    dr = DR.relation_mask(seed, rate, B, N)
    do = DR.object_mask(seed, rate, B, N)
    loss, logits, grads = O.loss_and_grads(params, objects, Rs, Rr, prop, target, S, drop_r=dr, drop_o=do)
    rec = dict(objects=objects, Rs=Rs.astype(np.float32), Rr=Rr.astype(np.float32), prop=prop, target=target,
               mp_steps=np.int32(S), logits=logits, loss=np.float64(loss), seed=np.uint64(seed), rate=np.float32(rate),
               drop_r_sum=np.float64(dr.sum()), drop_o_sum=np.float64(do.sum()))
    for k, g in grads.items():
        rec["grad/" + k] = g.astype(np.float64)
    np.savez_compressed(os.path.join(OUT, "golden_dropout_N6_B2_S5.npz"), **rec)
    print("wrote dropout fixture, loss", loss)


if __name__ == "__main__":
    main()
