"""bench.py's rank launcher on the GPU box (the driver runs `python3 bench.py
--gpus N` as is): N = 1 is one process on cuda:0; N = 2 on a box with fewer
GPUs than ranks must fail loudly instead of measuring one GPU."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(args):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK",
                                                            "GAC_BENCH_ONE_GPU")}
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py")] + args, capture_output=True,
                       text=True, timeout=240, env=env)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    return r, (json.loads(lines[-1]) if lines else None)


def test_bench_launch_one_gpu():
    r, out = _bench(["--gpus", "1", "--launch-check"])
    assert r.returncode == 0, r.stderr[-2000:]
    assert out["n_gpus"] == 1


def test_bench_launch_two_ranks():
    import torch
    r, out = _bench(["--gpus", "2", "--launch-check"])
    if torch.cuda.device_count() >= 2:
        assert r.returncode == 0, r.stderr[-2000:]
        g = out["process_group"]
        assert out["n_gpus"] == 2 and g["world_size"] == 2 and g["backend"] == "nccl"
        assert sorted(x["local_rank"] for x in g["ranks"]) == [0, 1]
    else:
        assert r.returncode != 0 and out is None
        assert "GPUs visible" in r.stderr, r.stderr[-2000:]
