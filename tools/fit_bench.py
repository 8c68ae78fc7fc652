"""Keras front-end training throughput at the reference's own settings (main.py:92-98: batch 32,
validation_split 0.2, shuffle): towers/s of model.fit on synthetic 6-block towers (thresholded
relations), each step a replayed hipGraph and, for comparison, the same steps issued eagerly. usage: python tools/fit_bench.py [n_samples] [epochs]"""
import json
import sys
import time

import numpy as np
import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from spwgnn_amd import data as D  # noqa: E402
from spwgnn_amd.keras_api import PropagationNetwork  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
epochs = int(sys.argv[2]) if len(sys.argv) > 2 else 3
obj, Rs, Rr, prop, tgt = D.synthetic_batch(n, 6, seed=3, fully_connected=False)
x = {"objects": obj, "sender_relations": Rs, "receiver_relations": Rr, "propagation": prop}
y = {"target": tgt.reshape(n, 6, 1)}
out = {}
for graph in (True, False):
    model = PropagationNetwork().getModel(6)
    model.fit(x, y, batch_size=32, epochs=1, validation_split=0.2, verbose=0, graph=graph)   # warm-up (+ capture)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    h = model.fit(x, y, batch_size=32, epochs=epochs, validation_split=0.2, verbose=0, graph=graph)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    n_tr = int(n * 0.8)
    steps = epochs * ((n_tr + 31) // 32)
    out["replayed" if graph else "eager"] = {
        "fit_towers_per_s": round(epochs * n_tr / el, 1), "ms_per_step": round(el / steps * 1e3, 3), "steps": steps,
        "losses": [round(v, 7) for v in h["loss"]]}
out["same_losses"] = out["replayed"]["losses"] == out["eager"]["losses"]
print(json.dumps(out))
