"""Multi-GPU sharding of one batch of sub-chain ranges or of a whole chain
set.

Chains / fills are independent, so a batch is split into contiguous shards
balanced by window blocks, each rank scores its shard on its own GPU, and a
single all-gather (RCCL over xGMI with backend "nccl"; gloo on CPU for tests)
reassembles the per-range results in input order -- the only collective on
the path.  One process per GPU (torch.distributed); rank r uses
cuda:LOCAL_RANK.  On GPUs everything stays in HBM: the shard's ranges, the
libgachain outputs (written straight into torch tensors by
gac_score_ranges_device on torch's current stream) and the gathered result.

The command-line tools split differently (no collective at all): chainNet
-nranks deals out chromosome sides, scoreChain -nranks contiguous chain runs
(their outputs are the exchange).  This module is for callers that hold one
range batch -- e.g. a rescoring service -- across the GPUs of a node, and
for scoreChain's batch in the north-star form (chain-ID shards + one RCCL
all-gather of {global, local, ali}), which bench.py measures at N > 1.
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


def gather_sharded(dist, world: int, n: int, bounds, local):
    """All-gather per-shard result rows (int64 tensor [rows, k], on the
    process group's device) into [n, k] in input order, on that device.
    Shards are padded to the largest one so one all_gather_into_tensor call
    (a single ring all-gather) moves everything; the padding is dropped by a
    gather on the same device (no host round trip)."""
    import torch
    k = local.shape[1]
    dev = local.device
    maxrows = max(hi - lo for lo, hi in bounds)
    buf = torch.zeros((maxrows, k), dtype=torch.int64, device=dev)
    if local.shape[0]:
        buf[: local.shape[0]] = local
    out = torch.empty((world * maxrows, k), dtype=torch.int64, device=dev)
    dist.all_gather_into_tensor(out, buf)
    idx = torch.cat([torch.arange(r * maxrows, r * maxrows + (hi - lo), device=dev)
                     for r, (lo, hi) in enumerate(bounds)])
    return out.index_select(0, idx) if n else out[:0]


def score_sharded(dist, rank: int, world: int, ranges: np.ndarray, weights: np.ndarray,
                  scorer: Callable, device=None):
    """Score `ranges` across all ranks.  scorer(shard_ranges) -> (global,
    local, ali) for this rank's shard (numpy, e.g. a CPU scorer in tests).
    Returns the full (global, local, ali) as numpy on every rank."""
    import torch
    bounds = shard_bounds(weights, world)
    lo, hi = bounds[rank]
    g, l, a = scorer(ranges[lo:hi])
    cols = (np.stack([np.asarray(g, np.int64), np.asarray(l, np.int64),
                      np.asarray(a, np.int64)], 1) if hi > lo else np.zeros((0, 3), np.int64))
    full = gather_sharded(dist, world, len(ranges), bounds,
                          torch.from_numpy(cols).to(device if device is not None else "cpu"))
    full = full.cpu().numpy()
    return full[:, 0], full[:, 1], full[:, 2].astype(np.int32)


def score_sharded_gpu(dist, rank: int, world: int, engine, chainset, ranges, weights,
                      want_local: bool = True):
    """The GPU path: `ranges` is an int32 [n, 3] torch tensor (or array) of
    (chain, tStart, tEnd) over a chain set every rank holds (`chainset`,
    uploaded to this rank's GPU by `engine`).  This rank's shard is scored by
    libgachain (gac_score_ranges_device) into device tensors on torch's
    current stream, then one all-gather over RCCL.  Returns an int64 [n, 3]
    device tensor (global, local, ali) on every rank."""
    import torch
    dev = torch.device("cuda", torch.cuda.current_device())
    r = torch.as_tensor(ranges, dtype=torch.int32)
    bounds = shard_bounds(np.asarray(weights), world)
    lo, hi = bounds[rank]
    m = hi - lo
    shard = r[lo:hi].to(dev).contiguous()
    g = torch.empty(m, dtype=torch.int64, device=dev)
    l = torch.empty(m, dtype=torch.int64, device=dev)
    a = torch.empty(m, dtype=torch.int32, device=dev)
    if m:
        engine.score_ranges_device(chainset, shard.data_ptr(), m, g.data_ptr(), a.data_ptr(),
                                   d_l=l.data_ptr() if want_local else 0, want_local=want_local,
                                   stream=torch.cuda.current_stream().cuda_stream)
    if not want_local:
        l.zero_()
    local = torch.stack([g, l, a.to(torch.int64)], 1)
    return gather_sharded(dist, world, r.shape[0], bounds, local)


def score_chains_sharded(dist, rank: int, world: int, n: int, weights: np.ndarray,
                         scorer: Callable, device=None):
    """scoreChain's batch across ranks: chain-ID shards --
    contiguous runs of chains balanced by `weights` (their block counts) --
    scored by scorer(lo, hi) -> (global, local, ali) of chains [lo, hi) on
    this rank, then ONE all-gather of {global, local, ali} reassembles the
    set in chain order on every rank.  Returns numpy (global, local, ali)."""
    import torch
    bounds = shard_bounds(weights, world)
    lo, hi = bounds[rank]
    g, l, a = scorer(lo, hi) if hi > lo else (np.zeros(0),) * 3
    cols = (np.stack([np.asarray(g, np.int64), np.asarray(l, np.int64),
                      np.asarray(a, np.int64)], 1) if hi > lo else np.zeros((0, 3), np.int64))
    full = gather_sharded(dist, world, n, bounds,
                          torch.from_numpy(cols).to(device if device is not None else "cpu"))
    full = full.cpu().numpy()
    return full[:, 0], full[:, 1], full[:, 2].astype(np.int32)


def score_chains_sharded_gpu(dist, rank: int, world: int, engine, shard_set, n: int, bounds,
                             want_local: bool = True):
    """The GPU path of score_chains_sharded: `shard_set` is this rank's chains
    [bounds[rank]) uploaded to its GPU; libgachain scores them whole
    (gac_score_chains_device) into device tensors on torch's current stream,
    and one all-gather over RCCL (xGMI) reassembles the int64 [n, 3]
    (global, local, ali) set on every rank's device."""
    import torch
    dev = torch.device("cuda", torch.cuda.current_device())
    lo, hi = bounds[rank]
    m = hi - lo
    g = torch.empty(m, dtype=torch.int64, device=dev)
    l = torch.zeros(m, dtype=torch.int64, device=dev)
    a = torch.empty(m, dtype=torch.int32, device=dev)
    if m:
        engine.score_chains_device(shard_set, g.data_ptr(), a.data_ptr(),
                                   d_l=l.data_ptr() if want_local else 0, want_local=want_local,
                                   stream=torch.cuda.current_stream().cuda_stream)
    local = torch.stack([g, l, a.to(torch.int64)], 1)
    return gather_sharded(dist, world, n, bounds, local)


def reduce_time_and_work(dist, seconds: float, work: float, device=None) -> Tuple[float, float]:
    """(max seconds over ranks, sum of work over ranks) -- bench.py's clock."""
    import torch
    t = torch.tensor([seconds, work], dtype=torch.float64, device=device)
    mx = t.clone()
    dist.all_reduce(mx, op=dist.ReduceOp.MAX)
    sm = t.clone()
    dist.all_reduce(sm, op=dist.ReduceOp.SUM)
    return float(mx[0]), float(sm[1])
