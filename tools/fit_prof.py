"""Host-side profile of Keras fit at batch 32 (replayed steps): cProfile of model.fit over the same
synthetic workload as tools/fit_bench.py, top functions by own time and cumulative time.
usage: python tools/fit_prof.py [n_samples] [epochs]"""
import cProfile
import os
import pstats
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from spwgnn_amd import data as D  # noqa: E402
from spwgnn_amd.keras_api import PropagationNetwork  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
epochs = int(sys.argv[2]) if len(sys.argv) > 2 else 3
obj, Rs, Rr, prop, tgt = D.synthetic_batch(n, 6, seed=3, fully_connected=False)
x = {"objects": obj, "sender_relations": Rs, "receiver_relations": Rr, "propagation": prop}
y = {"target": tgt.reshape(n, 6, 1)}
model = PropagationNetwork().getModel(6)
model.fit(x, y, batch_size=32, epochs=1, validation_split=0.2, verbose=0)
torch.cuda.synchronize()
pr = cProfile.Profile()
pr.enable()
model.fit(x, y, batch_size=32, epochs=epochs, validation_split=0.2, verbose=0)
torch.cuda.synchronize()
pr.disable()
st = pstats.Stats(pr)
st.sort_stats("tottime").print_stats(25)
st.sort_stats("cumulative").print_stats(30)
