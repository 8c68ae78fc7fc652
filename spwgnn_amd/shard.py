"""Shard planning for data-parallel training over ragged tower batches.

The reference trains one process on one batch (src/main.py:92-98); its loss is the mean BCE over
every node of the batch (`binary_crossentropy`, src/Networks.py:102). Data parallelism splits the
towers over ranks (towers are independent graphs: no halo, no data-path collective); balancing
must follow the work, which for ragged towers is dominated by the relations (∝ N(N−1)), not by the
tower count. The cost of a tower is the algorithmic MAC count of SURVEY §8d:

    fwd_MACs(N, E, S) = E·67,800 + N·10,200 + E·22,500 + S·(N·70,100 + E·37,500)

(the backward is ≈ 2× the forward for every term, so the forward count ranks the same).

`plan_shards` cuts the batch into `world` contiguous tower ranges at the quantiles of the cost
prefix sum: every rank's cost is within one tower's cost of total/world, tower order is kept (a
shard is a slice of the caller's batch), and the plan is a pure function of the sizes, so every
rank computes the same plan without communication.
"""
from __future__ import annotations

from typing import List, Tuple

import numpy as np

EDGE_MACS_ONCE = 67_800 + 22_500     # rm chain + the c_r·W1a term of rmp.0, once per relation
NODE_MACS_ONCE = 10_200              # om chain
EDGE_MACS_STEP = 37_500              # W2 row + the factored gathers, per relation per step
NODE_MACS_STEP = 70_100              # W3 + omp + U/V, per node per step


def tower_cost(tower_nodes, tower_edges, mp_steps: int = 5) -> np.ndarray:
    """Algorithmic forward MACs per tower (int64), SURVEY §8d."""
    n = np.asarray(tower_nodes, np.int64)
    e = np.asarray(tower_edges, np.int64)
    return e * EDGE_MACS_ONCE + n * NODE_MACS_ONCE + mp_steps * (n * NODE_MACS_STEP + e * EDGE_MACS_STEP)


def plan_shards(tower_nodes, tower_edges, world: int, mp_steps: int = 5) -> List[Tuple[int, int]]:
    """`world` contiguous [start, end) tower ranges of near-equal algorithmic cost.

    Rank r's range ends at the first tower whose cost prefix reaches (r+1)/world of the total, so
    |cost_r − total/world| ≤ max tower cost. Ranges may be empty only when there are fewer towers
    than ranks."""
    if world < 1:
        raise ValueError("world must be ≥ 1")
    cost = tower_cost(tower_nodes, tower_edges, mp_steps)
    T = len(cost)
    if T == 0:
        raise ValueError("empty batch: at least one tower is needed")
    cum = np.cumsum(cost)
    total = int(cum[-1])
    bounds = [0]
    for r in range(1, world):
        target = total * r / world
        # first index whose inclusive prefix passes the target; take the closer side of that tower
        i = int(np.searchsorted(cum, target, side="left"))
        lo = int(cum[i - 1]) if i > 0 else 0
        cut = i if (target - lo) <= (int(cum[i]) - target) else i + 1
        bounds.append(min(max(cut, bounds[-1]), T))
    bounds.append(T)
    return [(bounds[r], bounds[r + 1]) for r in range(world)]


def shard_weights(tower_nodes, ranges: List[Tuple[int, int]]) -> np.ndarray:
    """Per-rank node fraction n_r / n_global: the factor that turns a rank's mean-over-its-nodes
    BCE gradient into its share of the global mean (Σ_r w_r·g_r = ∇ mean over all B·N nodes)."""
    n = np.asarray(tower_nodes, np.int64)
    tot = int(n.sum())
    return np.array([n[a:b].sum() / tot for a, b in ranges], np.float64)


def micro_batches(start: int, end: int, max_towers: int) -> List[Tuple[int, int]]:
    """Split [start, end) into consecutive micro-batches of at most `max_towers` towers (config 4:
    a 2^17-tower shard trained as two micro-batches of 65,536 whose gradients are accumulated)."""
    if max_towers < 1:
        raise ValueError("max_towers must be ≥ 1")
    return [(a, min(a + max_towers, end)) for a in range(start, end, max_towers)]
