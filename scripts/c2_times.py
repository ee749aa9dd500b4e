"""C2 (configs[1]) end-to-end timing on the GPU box: bin/chainNet -rescore on
bench.py's C2 files, N runs, each run's wall and its device-open laps.
Usage: python scripts/c2_times.py [N]"""
import os
import subprocess
import sys
import time
import types

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    args = types.SimpleNamespace(tmp=os.environ.get("TMPDIR", "/tmp"), c2_chains=200_000)
    d, info = bench.c2_files(args)
    out = os.path.join(d, "ours")
    cmd = bench.tool_cmd(d, out, 1, 0)
    for i in range(n):
        for o in (out + ".t.net", out + ".q.net"):
            if os.path.exists(o):
                os.remove(o)
        t0 = time.perf_counter()
        r = subprocess.run(cmd, capture_output=True, text=True, env=dict(os.environ, GAC_TIMING="1"))
        dt = time.perf_counter() - t0
        laps = [ln for ln in r.stderr.splitlines() if ln.startswith(("[gac_open]", "[stage] fill", "[stage] (over"))]
        print(f"run {i}: {dt * 1e3:.1f} ms rc {r.returncode} | " + " | ".join(x.strip() for x in laps), flush=True)


if __name__ == "__main__":
    main()
