"""Multi-GPU sharding of one batch of sub-chain ranges.

Chains / fills are independent, so a batch is split into contiguous shards
balanced by window blocks, each rank scores its shard on its own GPU, and a
single all-gather (RCCL over xGMI with backend "nccl"; gloo on CPU for tests)
reassembles the per-range results in input order -- the only collective on
the path.  One process per GPU (torch.distributed); rank r uses cuda:LOCAL_RANK.
"""
from __future__ import annotations

from typing import Callable, List, Tuple

import numpy as np


def shard_bounds(weights: np.ndarray, world: int) -> List[Tuple[int, int]]:
    """Contiguous [lo, hi) shards of len(weights) items with ~equal weight."""
    n = len(weights)
    if world <= 1 or n == 0:
        return [(0, n)] + [(n, n)] * max(0, world - 1)
    cum = np.cumsum(np.asarray(weights, np.float64))
    total = cum[-1] if cum[-1] > 0 else 1.0
    cuts = [0]
    for r in range(1, world):
        cuts.append(int(np.searchsorted(cum, total * r / world, side="left")))
    cuts.append(n)
    for i in range(1, len(cuts)):  # monotone
        cuts[i] = max(cuts[i], cuts[i - 1])
    return [(cuts[i], cuts[i + 1]) for i in range(world)]


def gather_sharded(dist, rank: int, world: int, n: int, bounds, local_cols: np.ndarray,
                   device=None) -> np.ndarray:
    """All-gather per-shard result rows (int64 [rows, k]) into [n, k] in order.
    Shards are padded to the largest one so one all_gather_into_tensor call
    (a single ring all-gather) moves everything."""
    import torch
    k = local_cols.shape[1]
    maxrows = max(hi - lo for lo, hi in bounds)
    buf = torch.zeros((maxrows, k), dtype=torch.int64, device=device)
    if local_cols.shape[0]:
        buf[: local_cols.shape[0]] = torch.from_numpy(np.ascontiguousarray(local_cols)).to(device)
    out = torch.empty((world * maxrows, k), dtype=torch.int64, device=device)
    dist.all_gather_into_tensor(out, buf)
    out = out.cpu().numpy()
    res = np.empty((n, k), np.int64)
    for r, (lo, hi) in enumerate(bounds):
        res[lo:hi] = out[r * maxrows: r * maxrows + (hi - lo)]
    return res


def score_sharded(dist, rank: int, world: int, ranges: np.ndarray, weights: np.ndarray,
                  scorer: Callable[[np.ndarray], Tuple[np.ndarray, np.ndarray, np.ndarray]],
                  device=None):
    """Score `ranges` across all ranks.  scorer(shard_ranges) -> (global,
    local, ali) for this rank's shard (on its GPU).  Returns the full
    (global, local, ali) on every rank."""
    bounds = shard_bounds(weights, world)
    lo, hi = bounds[rank]
    g, l, a = scorer(ranges[lo:hi])
    cols = np.stack([np.asarray(g, np.int64), np.asarray(l, np.int64),
                     np.asarray(a, np.int64)], 1) if hi > lo else np.zeros((0, 3), np.int64)
    full = gather_sharded(dist, rank, world, len(ranges), bounds, cols, device)
    return full[:, 0], full[:, 1], full[:, 2].astype(np.int32)


def reduce_time_and_work(dist, seconds: float, work: float, device=None) -> Tuple[float, float]:
    """(max seconds over ranks, sum of work over ranks) -- bench.py's clock."""
    import torch
    t = torch.tensor([seconds, work], dtype=torch.float64, device=device)
    mx = t.clone()
    dist.all_reduce(mx, op=dist.ReduceOp.MAX)
    sm = t.clone()
    dist.all_reduce(sm, op=dist.ReduceOp.SUM)
    return float(mx[0]), float(sm[1])
