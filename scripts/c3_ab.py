"""C3 chainCleaner A/B on the GPU box: bin/chainCleaner on bench.py's C3 set
with GAC_CLEANER_SPEC=0 (round 5's batching) and =1 (speculative keys +
prefetch at a list's first pass), alternating; wall per run, the tool's GPU
call counts, and the outputs compared with each other and with the
reference's (run once).  Usage: python scripts/c3_ab.py OUTDIR [REPS]"""
import filecmp
import json
import os
import subprocess
import sys
import time
import types

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    out = sys.argv[1]
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    os.makedirs(out, exist_ok=True)
    d, info = bench.c3_files(types.SimpleNamespace(tmp=os.environ.get("TMPDIR", "/tmp")))
    p = lambda x: os.path.join(d, x)
    opts = [f"-net={p('in.net')}", "-linearGap=loose"]
    res = {"info": info, "runs": []}
    ref = [p("ref.chain"), p("ref.bed")]
    if os.path.exists(bench.REF_CC_TOOL) and not os.path.exists(ref[1]):
        env = dict(os.environ, PATH=os.path.dirname(bench.REF_CC_TOOL) + os.pathsep + os.environ["PATH"])
        subprocess.run([bench.REF_CC_TOOL, p("in.chain"), p("t.2bit"), p("q.2bit")] + ref + opts,
                       check=True, capture_output=True, env=env, timeout=300)
    for r in range(reps):
        for spec in os.environ.get("C3_MODES", "0 1").split():
            outs = [p(f"o{spec.replace(':', '_')}.chain"), p(f"o{spec.replace(':', '_')}.bed")]
            for o in outs:
                if os.path.exists(o):
                    os.remove(o)
            sp, _, la = spec.partition(":")  # "1:32": speculation on, 32 lists per batch
            env = dict(os.environ, GAC_CLEANER_SPEC=sp, GAC_TIMING="1")
            if la:
                env["GAC_CLEANER_LOOKAHEAD"] = la
            t0 = time.perf_counter()
            x = subprocess.run([bench.CC_TOOL, p("in.chain"), p("t.2bit"), p("q.2bit")] + outs + opts
                               + ["-verbose=2"], capture_output=True, text=True, env=env, timeout=300)
            dt = time.perf_counter() - t0
            assert x.returncode == 0, x.stderr[-2000:]
            lines = [ln for ln in x.stderr.splitlines() if ln.startswith(("GPU:", "host:", "[stage] 4", "[stage] 1"))]
            same_ref = (filecmp.cmp(outs[0], ref[0], False) and filecmp.cmp(outs[1], ref[1], False)
                        if os.path.exists(ref[1]) else None)
            res["runs"].append({"spec": spec, "rep": r, "wall_s": dt, "identical_to_reference": same_ref,
                                "stages": lines})
            print(spec, r, f"{dt:.3f}", same_ref, " | ".join(lines), flush=True)
    with open(os.path.join(out, "c3_ab.json"), "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
