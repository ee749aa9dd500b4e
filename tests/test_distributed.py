"""Multi-rank paths on CPU with gloo (world_size 2): sharding of one range
batch + the single all-gather that reassembles results in input order, and
bench.py's max-over-ranks clock.  The per-shard scorer here is the CPU oracle
(test-only); on GPUs it is libgachain behind the same callback."""
import os

import numpy as np
import pytest

from conftest import BLASTZ, GOLDEN


def test_shard_bounds():
    from genomealignmenttools_amd.shard import shard_bounds
    w = np.array([5, 1, 1, 1, 10, 1, 1, 1], float)
    b = shard_bounds(w, 2)
    assert b[0][0] == 0 and b[-1][1] == len(w) and b[0][1] == b[1][0]
    assert shard_bounds(w, 1) == [(0, len(w))]
    b8 = shard_bounds(np.ones(3), 8)
    assert sum(hi - lo for lo, hi in b8) == 3
    assert all(b8[i][1] == b8[i + 1][0] for i in range(7))


def _worker(rank, world, port, q):
    import torch.distributed as dist

    from genomealignmenttools_amd.chainfile import read_chains
    from genomealignmenttools_amd.shard import (reduce_time_and_work, score_chains_sharded,
                                                score_sharded)
    from oracle.oracle import OracleScorer, read_2bit_text
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        d = os.path.join(GOLDEN, "synth11")
        z = np.load(os.path.join(d, "subchain.npz"))
        ca = read_chains(os.path.join(d, "in.chain"))
        sc = OracleScorer(read_2bit_text(os.path.join(d, "t.2bit")),
                          read_2bit_text(os.path.join(d, "q.2bit")), BLASTZ, "loose")
        R = z["ranges"]
        w = np.diff(ca.blk_off)[R[:, 0]].astype(float)
        g, l, a = score_sharded(dist, rank, world, R, w, lambda r: sc.score_ranges(ca, r))
        ok = (np.array_equal(g, z["glob"]) and np.array_equal(l, z["loc"])
              and np.array_equal(a, z["ali"]))
        # whole chains (scoreChain's batch): chain-ID shards + one all-gather
        full = np.stack([np.arange(ca.n), ca.tstart, ca.tend], 1).astype(np.int64)
        og, ol, oa = sc.score_ranges(ca, full)
        g, l, a = score_chains_sharded(dist, rank, world, ca.n, np.diff(ca.blk_off).astype(float),
                                       lambda lo, hi: sc.score_ranges(ca, full[lo:hi]))
        ok = ok and np.array_equal(g, og) and np.array_equal(l, ol) and np.array_equal(a, oa)
        mx, sm = reduce_time_and_work(dist, 1.0 + rank, 10.0 * (rank + 1))
        q.put((rank, ok, mx, sm))
    finally:
        dist.destroy_process_group()


def test_gloo_world2_sharded_scoring():
    import socket

    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    for rank, ok, mx, sm in res:
        assert ok, f"rank {rank}: gathered results differ from the reference"
        assert mx == 2.0 and sm == 30.0
