"""Per-step kernel time vs wall time from a rocprofv3 --kernel-trace CSV of tools/fit_bench.py:
splits the trace at each step's first kernel (k_step_advance, or k_prep when the replayed step folds
its upload and key advance into the forward's first launch, spwgnn_run.prologue) and prints the median busy time per step
(union of kernel intervals), the median wall time from one step's first kernel start to the next
one's, the idle difference, and the median gap between consecutive launches.
usage: python tools/step_gaps.py TRACE_DIR"""
import csv
import glob
import sys

import numpy as np

path = glob.glob(f"{sys.argv[1]}/**/*kernel_trace.csv", recursive=True)[0]
rows = []
with open(path) as f:
    for r in csv.DictReader(f):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
rows.sort()
marker = "k_step_advance" if any("k_step_advance" in r[2] for r in rows) else "k_prep"
starts = [i for i, r in enumerate(rows) if marker in r[2]]
steps = [rows[a:b] for a, b in zip(starts, starts[1:])]
busy, wall, gaps = [], [], []
for s, nxt in zip(steps, steps[1:]):
    end, b = s[0][0], 0
    for a, e, _ in s:
        if a > end:
            gaps.append(a - end)
        b += max(0, e - max(a, end))
        end = max(end, e)
    busy.append(b)
    wall.append(nxt[0][0] - s[0][0])
busy, wall, gaps = np.array(busy), np.array(wall), np.array(gaps)
keep = wall < 2 * np.median(wall)     # drop the steps that straddle a validation pass or an epoch end
print(f"steps {keep.sum()} of {len(wall)}  launches/step {np.mean([len(s) for s in steps]):.1f}  "
      f"wall {np.median(wall[keep]) / 1e3:.1f} µs  busy {np.median(busy[keep]) / 1e3:.1f} µs  "
      f"idle {np.median((wall - busy)[keep]) / 1e3:.1f} µs  median gap between launches {np.median(gaps) / 1e3:.2f} µs")
# where the idle time sits: before the step's first launch (the batch upload) vs inside the step
lead = np.array([nxt[0][0] - max(e for _, e, _ in s) for s, nxt in zip(steps, steps[1:])])
names = {}
for s in steps[1:-1]:
    end = s[0][1]
    for a, e, n in s[1:]:
        names.setdefault(n.split("(")[0][-40:], []).append(a - end)
        end = max(end, e)
print(f"idle between steps (last kernel end -> next step's first start): median {np.median(lead[keep]) / 1e3:.1f} µs")
for n, g in sorted(names.items(), key=lambda kv: -np.median(kv[1]))[:6]:
    print(f"  gap before {n:42s} median {np.median(g) / 1e3:6.2f} µs")
