#!/usr/bin/env python3
"""Probe (measurement only): config C3 at hg38.mm10.chr1 scale -- the
inputs of tests/test_gpu_configs.py::test_c3_chaincleaner, then
bin/chainCleaner -net= with GAC_TIMING stage laps and the reference
chainCleaner on the same files, both timed.  Usage: c3_probe.py OUTDIR"""
import os
import subprocess
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
BIN = os.path.join(REPO, "genomealignmenttools_amd", "bin")
REF = os.path.join(REPO, "oracle", "_ref")


def run(cmd, **kw):
    t0 = time.time()
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=900, **kw)
    if r.returncode != 0:
        raise SystemExit(f"{cmd[0]} rc={r.returncode}: {r.stderr[-2000:]}")
    return r, time.time() - t0


def main():
    from genomealignmenttools_amd import chainfile, synth
    out = sys.argv[1]
    d = os.path.join(os.environ.get("TMPDIR", "/tmp"), "c3probe")
    os.makedirs(d, exist_ok=True)
    p = lambda x: os.path.join(d, x)
    t0 = time.time()
    tg, qg, ca = synth.c3_case(seed=42, n_chains=200_000, n_loci=1000)
    synth.write_2bit(tg, p("t.2bit"))
    synth.write_2bit(qg, p("q.2bit"))
    synth.write_sizes(tg.sizes, p("t.sizes"))
    synth.write_sizes(qg.sizes, p("q.sizes"))
    chainfile.write_chains_fast(ca, p("unscored.chain"))
    del tg, qg, ca
    run([os.path.join(BIN, "scoreChain"), p("unscored.chain"), p("t.2bit"), p("q.2bit"),
         p("sc.chain"), "-linearGap=loose"])
    sc = chainfile.read_chains(p("sc.chain"))
    sc = sc.subset(np.argsort(-sc.score, kind="stable"))
    sc.id = np.arange(1, sc.n + 1, dtype=np.int64)
    chainfile.write_chains_fast(sc, p("in.chain"))
    del sc
    net, _ = run([os.path.join(REF, "chainNet"), "-minScore=0", p("in.chain"), p("t.sizes"),
                  p("q.sizes"), "stdout", "/dev/null"])
    filt = subprocess.run([os.path.join(BIN, "NetFilterNonNested.perl"), "/dev/stdin",
                           "-minScore1", "3000"], input=net.stdout, capture_output=True,
                          text=True, timeout=600)
    with open(p("in.net"), "w") as f:
        f.write(filt.stdout)
    print(f"inputs {time.time() - t0:.1f}s", flush=True)
    opts = [f"-net={p('in.net')}", "-linearGap=loose"]
    lines = []
    for k in range(3):
        r, dt = run([os.path.join(BIN, "chainCleaner"), p("in.chain"), p("t.2bit"), p("q.2bit"),
                     p("ours.chain"), p("ours.bed")] + opts + (["-verbose=2"] if k == 2 else []),
                    env=dict(os.environ, GAC_TIMING="1") if k == 2 else None)
        lines.append(f"ours run {k}: {dt:.3f} s")
        if k == 2:
            lines += [x for x in r.stderr.splitlines() if x.startswith("[")]
    env = dict(os.environ, PATH=REF + os.pathsep + os.environ["PATH"])
    _, dt = run([os.path.join(REF, "chainCleaner"), p("in.chain"), p("t.2bit"), p("q.2bit"),
                 p("ref.chain"), p("ref.bed")] + opts, env=env)
    same = open(p("ours.chain")).read() == open(p("ref.chain")).read() and \
        open(p("ours.bed")).read() == open(p("ref.bed")).read()
    lines.append(f"reference chainCleaner: {dt:.3f} s; outputs identical: {same}")
    with open(out, "w") as f:
        f.write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main()
