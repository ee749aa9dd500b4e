"""bench.py's CPU-baseline helpers (no GPU): splitting a chain file by target
sequence for the all-cores reference run, and the aligned-bases measure."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def _chain(score, t, q, blocks, cid):
    ts = 100
    lines = [f"chain {score} {t} 1000000 + {ts} {ts + sum(b[0] + b[1] for b in blocks)} "
             f"{q} 900000 + 50 {50 + sum(b[0] + b[2] for b in blocks)} {cid}"]
    for k, (size, dt, dq) in enumerate(blocks):
        lines.append(f"{size}" if k == len(blocks) - 1 else f"{size}\t{dt}\t{dq}")
    return "\n".join(lines) + "\n\n"


def test_split_by_target(tmp_path):
    import bench
    rng = np.random.default_rng(3)
    chains, want = [], {"chr7": [], "chr21": []}
    for i in range(301):  # (the last chain, on chr7, is kept)
        t = ["chr7", "chr21", "chr1", "chr21_alt"][i % 4]
        nb = int(rng.integers(1, 6))
        blocks = [(int(rng.integers(1, 50)), int(rng.integers(0, 30)), int(rng.integers(0, 30)))
                  for _ in range(nb)]
        blocks[-1] = (blocks[-1][0], 0, 0)
        txt = _chain(1000 - i, t, "chrQ", blocks, i + 1)
        chains.append(txt)
        if t in want:
            want[t].append(txt)
    src = tmp_path / "in.chain"
    src.write_text("#meta line\n" + "".join(chains))
    out = bench._split_by_target(str(src), ("chr7", "chr21"), str(tmp_path))
    for t in ("chr7", "chr21"):
        with open(out[t]) as f:
            assert f.read() == "".join(want[t])
