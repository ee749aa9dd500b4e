#!/usr/bin/env python3
"""Per-call latency of small batches (gac_score_ranges with n <= 256 and
gac_score_ranges_host), with and without the small-batch server.
usage: small_latency.py [CALLS] [N_RANGES]  (env GAC_SMALL_SERVER decides)"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from genomealignmenttools_amd import synth  # noqa: E402
from genomealignmenttools_amd.gachain import GAC_Q, GAC_T, Engine, GapCosts  # noqa: E402

BLASTZ = np.array([91, -114, -31, -123, -114, 100, -125, -31, -31, -125, 100, -114,
                   -123, -31, -114, 91], np.int32)


def main():
    calls = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
    nr = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    tg, qg, ca = synth.small_case(seed=23, n_chains=200, max_blocks=400, n_frac=0.05)
    e = Engine(0)
    e.add_sequences(GAC_T, tg.seq_records())
    e.add_sequences(GAC_Q, qg.seq_records())
    e.set_scoring(BLASTZ, GapCosts("loose"))
    cs = e.upload_chains(ca)
    tix = np.array([e.seq_index(GAC_T, x) for x in ca.tname], np.int32)
    qix = np.array([e.seq_index(GAC_Q, x) for x in ca.qname], np.int32)
    arrs = (tix, qix, ca.qstrand, ca.blk_off, ca.blk_t, ca.blk_q, ca.blk_size)
    rng = np.random.default_rng(1)
    c = rng.integers(0, ca.n, nr)
    R = np.stack([c, ca.tstart[c], ca.tend[c]], 1).astype(np.int32)
    for kind, fn in (("set", lambda: e.score_ranges(cs, R, want_local=True)),
                     ("host", lambda: e.score_ranges_host(*arrs, R, want_local=True)),
                     ("noop", lambda: e.seq_count(GAC_T))):
        for _ in range(50):
            fn()
        t0 = time.perf_counter()
        for _ in range(calls):
            fn()
        dt = (time.perf_counter() - t0) / calls * 1e6
        print(f"server={os.environ.get('GAC_SMALL_SERVER', '0')} {kind}: {dt:.1f} us per call "
              f"({nr} ranges)", flush=True)
    e.close()


if __name__ == "__main__":
    main()
