#!/usr/bin/env python3
"""A/B of bin/chainCleaner on C3 (bench.py's c3 files) under environment
variants, alternating, with the reference's outputs as the check.
usage: c3_ab.py [REPS] [tag:ENV=v,ENV2=v ...]   (default: base vs the small-batch server)"""
import filecmp
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.argv = [sys.argv[0]] + sys.argv[1:]
import bench  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    specs = sys.argv[2:] or ["base:GAC_SMALL_SERVER=0", "srv:GAC_SMALL_SERVER=1"]
    variants = []
    for sp in specs:
        tag, _, kv = sp.partition(":")
        env = dict(os.environ)
        for x in filter(None, kv.split(",")):
            k, _, v = x.partition("=")
            env[k] = v
        variants.append((tag, env))
    sys.argv = [sys.argv[0]]
    args = bench.parse()
    d, info = bench.c3_files(args)
    p = lambda x: os.path.join(d, x)
    opts = [f"-net={p('in.net')}", "-linearGap=loose"]
    ro = [p("ref.chain"), p("ref.bed")]
    if not all(os.path.exists(x) for x in ro):
        t0 = time.time()
        env = dict(os.environ, PATH=os.path.dirname(bench.REF_CC_TOOL) + os.pathsep + os.environ["PATH"])
        bench.run_tool([bench.REF_CC_TOOL, p("in.chain"), p("t.2bit"), p("q.2bit")] + ro + opts, ro,
                       env=env)
        print(f"reference: {time.time() - t0:.2f} s", flush=True)
    for rep in range(reps):
        for tag, env in variants:
            outs = [p(f"{tag}.chain"), p(f"{tag}.bed")]
            cmd = [bench.CC_TOOL, p("in.chain"), p("t.2bit"), p("q.2bit")] + outs + opts + ["-verbose=" + os.environ.get("C3_VERBOSE", "1")]
            e2 = dict(env, GAC_TIMING="1")
            t0 = time.perf_counter()
            r = bench.run_tool(cmd, outs, env=e2)
            dt = time.perf_counter() - t0
            same = all(filecmp.cmp(a, b, False) for a, b in zip(outs, ro))
            lines = [x.strip() for x in r.stderr.splitlines()
                     if x.startswith(("GPU", "[stage] 4.", "[stage] 1."))]
            print(f"{tag} rep {rep}: {dt * 1e3:.0f} ms identical={same} | " + " | ".join(lines),
                  flush=True)
            if not same:
                sys.exit(1)


if __name__ == "__main__":
    main()
