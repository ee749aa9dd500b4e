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


def _bench(args, env=None, timeout=300):
    import json
    import subprocess
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py")] + args, capture_output=True,
                       text=True, timeout=timeout, env=dict(os.environ, **(env or {})))
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    return r, (json.loads(lines[-1]) if lines else None)


def test_bench_self_launch_two_ranks():
    """`python bench.py --gpus 2` outside torchrun starts the two ranks itself
    (one torch.distributed.run child) and the line's n_gpus is the process
    group's size; here the ranks are the gloo rehearsal (GAC_BENCH_ONE_GPU)."""
    env = {"GAC_BENCH_ONE_GPU": "1"}
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        os.environ.pop(k, None)
    r, out = _bench(["--gpus", "2", "--launch-check"], env)
    assert r.returncode == 0, r.stderr[-2000:]
    assert out["n_gpus"] == 2
    g = out["process_group"]
    assert g["world_size"] == 2 and g["backend"] == "gloo"
    assert sorted(x["rank"] for x in g["ranks"]) == [0, 1]
    assert len({x["pid"] for x in g["ranks"]}) == 2


def test_bench_world_mismatch_fails():
    """A torchrun world that is not --gpus is an error, not a 1-GPU number."""
    r, out = _bench(["--gpus", "3", "--launch-check"], {"WORLD_SIZE": "2", "RANK": "0"})
    assert r.returncode != 0 and out is None
    assert "--gpus 3" in r.stderr


def test_launch_cmd():
    import bench
    cmd = bench.launch_cmd(8, ["--gpus", "8", "--steps", "3"], 29500)
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in cmd and "--master-addr=127.0.0.1" in cmd
    assert cmd[-4:] == ["--gpus", "8", "--steps", "3"]


def test_full_parity_helper(tmp_path):
    """bench.full_parity hashes the files against tests/golden/fullscale/*.json
    (both goldens hold the keys bench and the GPU tests read); a run on another
    seed or size (its input's sha differs from the golden's) reports parity
    unpinned instead of a mismatch."""
    import hashlib
    import json
    import bench
    for which, keys in (("c5", ["in_chain_sha256", "chainnet_rescore.t_net_sha256",
                                "chainnet_rescore.q_net_sha256", "scorechain.chain_sha256"]),
                        ("c4", ["in_psl_sha256", "axtchain.chain_sha256"])):
        files = {}
        for k in keys:
            f = tmp_path / f"{which}.{k}"
            f.write_bytes(k.encode() * 1000)
            files[k] = str(f)
        res = bench.full_parity(which, files)
        # an input that is not the golden's input: parity unpinned, not "False"
        assert res["identical"] is None and "unpinned" in res
        for k in keys:
            assert res[k]["ours"] == hashlib.sha256(k.encode() * 1000).hexdigest()
            assert len(res[k]["reference"]) == 64 and res[k]["same"] is False
        g = json.load(open(os.path.join(REPO, "tests", "golden", "fullscale", f"{which}.json")))
        assert g["info"]["seed"] in (7, 1234)


def test_rank_tool_threads(tmp_path):
    """N > 1: each rank's tool gets the node's usable CPUs shared by its
    ranks -- also under torch.distributed.run's default OMP_NUM_THREADS=1,
    which would otherwise run every rank's netting on one thread; a
    launcher's own GAC_THREADS / OMP_NUM_THREADS is kept; the cgroup quota
    narrows the CPU count."""
    import bench
    assert bench.rank_tool_threads(1, {}, 128) == {}
    assert bench.rank_tool_threads(8, {}, 128) == {"GAC_THREADS": "16"}
    tr = {"OMP_NUM_THREADS": "1", "TORCHELASTIC_RUN_ID": "x", "LOCAL_WORLD_SIZE": "4"}
    assert bench.rank_tool_threads(8, tr, 128) == {"GAC_THREADS": "32"}
    assert bench.rank_tool_threads(8, {"OMP_NUM_THREADS": "1"}, 128) == {}
    assert bench.rank_tool_threads(8, {"OMP_NUM_THREADS": "12", "TORCHELASTIC_RUN_ID": "x"}, 128) == {}
    assert bench.rank_tool_threads(8, {"GAC_THREADS": "3", **tr}, 128) == {}
    assert bench.rank_tool_threads(8, {}, 4) == {"GAC_THREADS": "1"}
    q = tmp_path / "cpu.max"
    q.write_text("1600000 100000\n")
    assert bench.usable_cpus(str(q)) == min(16, len(os.sched_getaffinity(0)))
    q.write_text("max 100000\n")
    assert bench.usable_cpus(str(q)) == len(os.sched_getaffinity(0))
