#!/usr/bin/env python3
"""End-to-end tool timings beside the reference binaries (SURVEY §8(d)
configs C3/C4), on the GPU box's own host.

  python scripts/bench_tools.py axtchain --blocks 5000000
  python scripts/bench_tools.py cleaner --loci 2000

axtchain: synth.psl_c4 (seeded C4-like PSL: power-law blocks per chromosome
pair, 80% planted collinear, 20% random), run by bin/axtChain and by the
reference axtChain compiled from /root/reference (oracle/_ref/axtChain,
test infrastructure; timed as the CPU baseline), outputs compared byte for
byte.  cleaner: synth.cleaner_case at scale, chainNet -minScore=0 + the
in-process filter via bin/chainCleaner without -net vs the reference
chainCleaner given the reference chainNet|NetFilterNonNested net (timed
separately).  Prints one JSON line per run; files go to --tmp.
"""
import argparse
import filecmp
import hashlib
import json
import os
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from genomealignmenttools_amd import chainfile, synth  # noqa: E402

BIN = os.path.join(REPO, "genomealignmenttools_amd", "bin")
REF = os.path.join(REPO, "oracle", "_ref")


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def timed(cmd, cwd=None, env=None, timeout=3000, outputs=()):
    # outputs are removed first: overwriting a file truncates it, and some
    # filesystems (ext4 auto_da_alloc) flush a truncated-and-rewritten file
    # on close, which would time the disk instead of the tool
    for o in outputs:
        if os.path.exists(o):
            os.remove(o)
    t = time.time()
    r = subprocess.run(cmd, capture_output=True, text=True, cwd=cwd, env=env, timeout=timeout)
    dt = time.time() - t
    if r.returncode != 0:
        raise RuntimeError(f"{cmd} failed rc={r.returncode}: {r.stderr[-3000:]}")
    return dt, r


def sha(path):
    h = hashlib.sha256()
    with open(path, "rb") as f:
        for b in iter(lambda: f.read(1 << 20), b""):
            h.update(b)
    return h.hexdigest()[:16]


def axtchain(a):
    d = os.path.join(a.tmp, f"c4_{a.blocks}")
    os.makedirs(d, exist_ok=True)
    psl = os.path.join(d, "in.psl")
    if not os.path.exists(psl):
        t = time.time()
        tg, qg, pairs, b = synth.psl_c4(a.seed, a.blocks, tsize=a.tsize, qsize=a.qsize)
        synth.write_2bit(tg, os.path.join(d, "t.2bit"))
        synth.write_2bit(qg, os.path.join(d, "q.2bit"))
        nrec = synth.write_psl_c4(tg, qg, pairs, b, psl, a.seed)
        log(f"generated {len(b['t'])} blocks, {nrec} records in {time.time() - t:.1f}s")
    env = dict(os.environ, GAC_TIMING="1", GAC_AXT_DP=a.dp)
    args = ["-psl", psl, os.path.join(d, "t.2bit"), os.path.join(d, "q.2bit")]
    ours = os.path.join(d, "ours.chain")
    t_ours, r = timed([os.path.join(BIN, "axtChain"), "-linearGap=loose", "-verbose=0"] + args +
                      [ours], env=env, outputs=[ours])
    log(r.stderr)
    res = {"tool": "axtChain", "blocks": a.blocks, "seed": a.seed, "dp": a.dp, "ours_s": round(t_ours, 3),
           "ours_sha": sha(ours), "timing": [l for l in r.stderr.splitlines() if "gac_axt" in l]}
    refbin = os.path.join(REF, "axtChain")
    if os.path.exists(refbin) and not a.no_ref:
        ref = os.path.join(d, "ref.chain")
        t_ref, _ = timed([refbin, "-linearGap=loose", "-verbose=0"] + args + [ref], outputs=[ref])
        res.update(ref_s=round(t_ref, 3), ref_cores=1, identical=filecmp.cmp(ours, ref, False),
                   speedup=round(t_ref / t_ours, 2))
    res["chains"] = sum(1 for line in open(ours) if line.startswith("chain"))
    print(json.dumps(res), flush=True)


def cleaner(a):
    d = os.path.join(a.tmp, f"c3_{a.loci}")
    os.makedirs(d, exist_ok=True)
    inc = os.path.join(d, "in.chain")
    if not os.path.exists(inc):
        t = time.time()
        tg, qg, chains = synth.cleaner_case(a.seed, a.loci)
        synth.write_2bit(tg, os.path.join(d, "t.2bit"))
        synth.write_2bit(qg, os.path.join(d, "q.2bit"))
        synth.write_sizes(tg.sizes, os.path.join(d, "t.sizes"))
        synth.write_sizes(qg.sizes, os.path.join(d, "q.sizes"))
        ca = synth.chains_to_arrays(tg, qg, chains)
        chainfile.write_chains(ca, os.path.join(d, "unscored.chain"))
        # header scores from our own scoreChain (byte-identical to the reference's)
        timed([os.path.join(BIN, "scoreChain"), os.path.join(d, "unscored.chain"),
               os.path.join(d, "t.2bit"), os.path.join(d, "q.2bit"), os.path.join(d, "sc.chain"),
               "-linearGap=loose"])
        sc = chainfile.read_chains(os.path.join(d, "sc.chain"))
        import numpy as np
        order = np.argsort(-sc.score, kind="stable")
        sc = sc.subset(order)
        sc.id = np.arange(1, sc.n + 1, dtype=np.int64)
        chainfile.write_chains(sc, inc)
        log(f"generated {sc.n} chains in {time.time() - t:.1f}s")
    p = lambda x: os.path.join(d, x)
    t_ours, r = timed([os.path.join(BIN, "chainCleaner"), inc, p("t.2bit"), p("q.2bit"),
                       p("ours.chain"), p("ours.bed"), f"-tSizes={p('t.sizes')}",
                       f"-qSizes={p('q.sizes')}", "-linearGap=loose", "-verbose=1"], cwd=d,
                      env=dict(os.environ, GAC_TIMING="1"), outputs=[p("ours.chain"), p("ours.bed")])
    res = {"tool": "chainCleaner", "loci": a.loci, "seed": a.seed, "ours_s": round(t_ours, 3),
           "removed": sum(1 for _ in open(p("ours.bed"))),
           "gpu": [l for l in r.stderr.splitlines() if l.startswith("GPU:")],
           "stages": [l for l in r.stderr.splitlines() if "[stage]" in l]}
    if os.path.exists(os.path.join(REF, "chainCleaner")) and not a.no_ref:
        env = dict(os.environ, PATH=REF + os.pathsep + os.environ.get("PATH", ""))
        t_net, rn = timed([os.path.join(REF, "chainNet"), "-minScore=0", inc, p("t.sizes"),
                           p("q.sizes"), "stdout", "/dev/null"])
        t0 = time.time()
        # the reference's perl filter when /root/reference is present (build
        # container), else the product's C port (bin/NetFilterNonNested)
        perl = "/root/reference/src/NetFilterNonNested.perl"
        filt = (["perl", perl] if os.path.exists(perl) else
                [os.path.join(BIN, "NetFilterNonNested.perl")])
        net = subprocess.run(filt + ["/dev/stdin", "-minScore1", "3000"], input=rn.stdout,
                             capture_output=True, text=True)
        res["ref_filter"] = "perl" if filt[0] == "perl" else "bin/NetFilterNonNested.perl"
        t_filter = time.time() - t0
        if net.returncode == 0:
            with open(p("ref.net"), "w") as f:
                f.write(net.stdout)
            t_ref, _ = timed([os.path.join(REF, "chainCleaner"), inc, p("t.2bit"), p("q.2bit"),
                              p("ref.chain"), p("ref.bed"), f"-net={p('ref.net')}",
                              "-linearGap=loose", "-verbose=0"], cwd=d, env=env,
                             outputs=[p("ref.chain"), p("ref.bed")])
            res.update(ref_s=round(t_net + t_filter + t_ref, 3), ref_net_s=round(t_net, 3),
                       ref_filter_s=round(t_filter, 3), ref_clean_s=round(t_ref, 3), ref_cores=1,
                       identical=filecmp.cmp(p("ours.chain"), p("ref.chain"), False)
                       and filecmp.cmp(p("ours.bed"), p("ref.bed"), False))
            res["speedup"] = round(res["ref_s"] / t_ours, 2)
        else:
            res["ref_error"] = "perl filter unavailable: " + net.stderr[-200:]
    print(json.dumps(res), flush=True)


def c2_files(a):
    """C2: hg38 chr1 x all mm10, ~2e5 planted chains, seed 42,
    written once under --tmp (2bit genomes, chrom.sizes, chains)."""
    d = os.path.join(a.tmp, f"c2_{a.chains}_{a.seed}")
    os.makedirs(d, exist_ok=True)
    if not os.path.exists(os.path.join(d, "in.chain")):
        t = time.time()
        tg, qg, ca = synth.c2_case(a.seed, a.chains)
        synth.write_2bit(tg, os.path.join(d, "t.2bit"))
        synth.write_2bit(qg, os.path.join(d, "q.2bit"))
        synth.write_sizes(tg.sizes, os.path.join(d, "t.sizes"))
        synth.write_sizes(qg.sizes, os.path.join(d, "q.sizes"))
        chainfile.write_chains(ca, os.path.join(d, "in.chain"))
        log(f"C2: {ca.n} chains, {ca.aligned_bases()} aligned bases, {time.time() - t:.1f}s")
    return d


def scorechain(a):
    d = c2_files(a)
    p = lambda x: os.path.join(d, x)
    args = [p("in.chain"), p("t.2bit"), p("q.2bit")]
    t_ours, r = timed([os.path.join(BIN, "scoreChain")] + args + [p("ours.chain"), "-linearGap=loose",
                                                                  "-verbose=2"],
                      outputs=[p("ours.chain")])
    res = {"tool": "scoreChain", "chains": a.chains, "seed": a.seed, "ours_s": round(t_ours, 3),
           "stages": [l for l in r.stderr.splitlines() if "[stage]" in l]}
    if os.path.exists(os.path.join(REF, "scoreChain")) and not a.no_ref:
        t_ref, _ = timed([os.path.join(REF, "scoreChain")] + args + [p("ref.chain"),
                                                                     "-linearGap=loose"],
                         outputs=[p("ref.chain")])
        res.update(ref_s=round(t_ref, 3), ref_cores=1, speedup=round(t_ref / t_ours, 2),
                   identical=filecmp.cmp(p("ours.chain"), p("ref.chain"), False))
    print(json.dumps(res), flush=True)


def chainnet(a):
    d = c2_files(a)
    p = lambda x: os.path.join(d, x)
    args = [p("in.chain"), p("t.sizes"), p("q.sizes")]
    opts = ["-rescore", f"-tNibDir={p('t.2bit')}", f"-qNibDir={p('q.2bit')}", "-linearGap=loose"]
    t_ours, r = timed([os.path.join(BIN, "chainNet")] + args + [p("ours.t.net"), p("ours.q.net")] +
                      opts + ["-verbose=2"], outputs=[p("ours.t.net"), p("ours.q.net")])
    res = {"tool": "chainNet -rescore", "chains": a.chains, "seed": a.seed,
           "ours_s": round(t_ours, 3),
           "stages": [l for l in r.stderr.splitlines() if "[stage]" in l]}
    if os.path.exists(os.path.join(REF, "chainNet")) and not a.no_ref:
        t_ref, _ = timed([os.path.join(REF, "chainNet")] + args + [p("ref.t.net"), p("ref.q.net")] +
                         opts, outputs=[p("ref.t.net"), p("ref.q.net")])
        res.update(ref_s=round(t_ref, 3), ref_cores=1, speedup=round(t_ref / t_ours, 2),
                   identical=filecmp.cmp(p("ours.t.net"), p("ref.t.net"), False)
                   and filecmp.cmp(p("ours.q.net"), p("ref.q.net"), False))
    print(json.dumps(res), flush=True)


def host_info():
    model = ""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {"host_cpu": model, "host_nproc": os.cpu_count(),
            "threads": int(os.environ.get("GAC_THREADS") or os.environ.get("OMP_NUM_THREADS") or 0)
            or os.cpu_count()}


def c5(a):
    """Whole-genome C5 (every hg38 x every mm10 sequence) at --chains chains:
    scoreChain and chainNet -rescore end to end, ours vs the reference
    binaries on this host, outputs compared byte for byte."""
    d = os.path.join(a.tmp, f"c5_{a.chains}_{a.seed}")
    os.makedirs(d, exist_ok=True)
    p = lambda x: os.path.join(d, x)
    gen_s = 0.0
    if not os.path.exists(p("in.chain")):
        t = time.time()
        tg, qg, ca = synth.c5_case(a.seed, a.chains)
        synth.write_2bit(tg, p("t.2bit"))
        synth.write_2bit(qg, p("q.2bit"))
        synth.write_sizes(tg.sizes, p("t.sizes"))
        synth.write_sizes(qg.sizes, p("q.sizes"))
        chainfile.write_chains(ca, p("in.chain.tmp"))
        os.rename(p("in.chain.tmp"), p("in.chain"))
        info = {"chains": ca.n, "blocks": int(len(ca.blk_size)), "aligned_bases": ca.aligned_bases(),
                "t_seqs": len(tg.names), "q_seqs": len(qg.names),
                "t_seqs_with_chains": len(set(ca.tname))}
        with open(p("info.json"), "w") as f:
            json.dump(info, f)
        del tg, qg, ca
        gen_s = time.time() - t
        log(f"C5: {info} generated in {gen_s:.1f}s")
    with open(p("info.json")) as f:
        info = json.load(f)
    res = {"tool": "C5 scoreChain + chainNet -rescore", "seed": a.seed, **info, **host_info(),
           "gen_s": round(gen_s, 1)}
    sc_args = [p("in.chain"), p("t.2bit"), p("q.2bit")]
    t1, r1 = timed([os.path.join(BIN, "scoreChain")] + sc_args + [p("ours.sc.chain"),
                                                                   "-linearGap=loose", "-verbose=2"],
                   outputs=[p("ours.sc.chain")])
    cn_args = [p("in.chain"), p("t.sizes"), p("q.sizes")]
    opts = ["-rescore", f"-tNibDir={p('t.2bit')}", f"-qNibDir={p('q.2bit')}", "-linearGap=loose"]
    t2, r2 = timed([os.path.join(BIN, "chainNet")] + cn_args + [p("ours.t.net"), p("ours.q.net")] +
                   opts + ["-verbose=2"], outputs=[p("ours.t.net"), p("ours.q.net")])
    res.update(ours_scorechain_s=round(t1, 3), ours_chainnet_s=round(t2, 3),
               ours_s=round(t1 + t2, 3),
               ours_stages=[l for l in (r1.stderr + r2.stderr).splitlines()
                            if "[stage]" in l or "[gac_chains_upload]" in l],
               ours_gbases_per_s=round(2 * info["aligned_bases"] / (t1 + t2) / 1e9, 3))
    log(f"ours: scoreChain {t1:.2f}s chainNet {t2:.2f}s")
    print(json.dumps(res), flush=True)  # ours alone, in case the reference run is cut off
    if os.path.exists(os.path.join(REF, "chainNet")) and not a.no_ref:
        # the two single-threaded reference tools run side by side (one core
        # each, timed separately): the C5 run then fits one GPU-box call
        import threading
        sc_res = {}
        th = threading.Thread(target=lambda: sc_res.update(t=timed(
            [os.path.join(REF, "scoreChain")] + sc_args + [p("ref.sc.chain"), "-linearGap=loose"],
            outputs=[p("ref.sc.chain")])[0]))
        th.start()
        t4, _ = timed([os.path.join(REF, "chainNet")] + cn_args + [p("ref.t.net"), p("ref.q.net")] +
                      opts, outputs=[p("ref.t.net"), p("ref.q.net")])
        th.join()
        t3 = sc_res["t"]
        log(f"ref scoreChain {t3:.2f}s, ref chainNet {t4:.2f}s (side by side)")
        res.update(ref_scorechain_s=round(t3, 3), ref_chainnet_s=round(t4, 3),
                   ref_s=round(t3 + t4, 3), ref_cores=1, speedup=round((t3 + t4) / (t1 + t2), 2),
                   identical={"scoreChain": filecmp.cmp(p("ours.sc.chain"), p("ref.sc.chain"), False),
                              "t.net": filecmp.cmp(p("ours.t.net"), p("ref.t.net"), False),
                              "q.net": filecmp.cmp(p("ours.q.net"), p("ref.q.net"), False)})
    print(json.dumps(res), flush=True)


def microjobs(a):
    """RepeatFiller-style micro-jobs: --jobs small
    axtChain runs (the reference's chrM known-answer alignment, each to its
    own output), as separate processes of the reference, separate processes
    of ours, and one `axtChain -jobs=FILE` batch; all outputs compared."""
    g = os.path.join(REPO, "tests", "golden", "chrM")
    d = os.path.join(a.tmp, "microjobs")
    os.makedirs(d, exist_ok=True)
    args = lambda out: ["-psl", os.path.join(g, "newStyleLastz.psl"), "-minScore=3000",
                        "-linearGap=loose", os.path.join(g, "hg19.chrM.2bit"),
                        "-scoreScheme=" + os.path.join(g, "newStyleLastz.Q.txt"),
                        os.path.join(g, "susScr3.chrM.2bit"), out]
    outs = lambda tag: [os.path.join(d, f"{tag}{i}.chain") for i in range(a.jobs)]
    res = {"tool": "axtChain micro-jobs", "jobs": a.jobs, "blocks_per_job": 0}
    if not a.no_separate:  # one process (one HIP bring-up) per job
        t = time.time()
        for o in outs("sep"):
            timed([os.path.join(BIN, "axtChain")] + args(o), outputs=[o])
        res["ours_separate_s"] = round(time.time() - t, 3)
    jobs = os.path.join(d, "jobs.txt")
    with open(jobs, "w") as f:
        for o in outs("bat"):
            f.write(" ".join(args(o)) + "\n")
    t_b, _ = timed([os.path.join(BIN, "axtChain"), f"-jobs={jobs}"], outputs=outs("bat"))
    res["ours_batch_s"] = round(t_b, 3)
    want = os.path.join(g, "newStyleLastz.chain")
    same = all(filecmp.cmp(o, want, False) for o in (outs("bat") if a.no_separate else
                                                      outs("sep") + outs("bat")))
    refbin = os.path.join(REF, "axtChain")
    if os.path.exists(refbin) and not a.no_ref:
        t = time.time()
        for o in outs("ref"):
            timed([refbin] + args(o), outputs=[o])
        res["ref_separate_s"] = round(time.time() - t, 3)
        same = same and all(filecmp.cmp(o, want, False) for o in outs("ref"))
        res["speedup_batch_vs_ref"] = round(res["ref_separate_s"] / t_b, 2)
    res["identical"] = same
    with open(os.path.join(g, "newStyleLastz.psl")) as f:
        res["blocks_per_job"] = sum(int(l.split()[17]) for l in f if l[:1].isdigit())
    print(json.dumps(res), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("tool", choices=["axtchain", "cleaner", "scorechain", "chainnet", "c5",
                                     "microjobs"])
    ap.add_argument("--jobs", type=int, default=200)
    ap.add_argument("--dp", choices=["host", "gpu"], default="host",
                    help="axtchain: kd-tree DP on host threads or on the device (GAC_AXT_DP)")
    ap.add_argument("--no-separate", action="store_true")
    ap.add_argument("--chains", type=int, default=200_000)
    ap.add_argument("--blocks", type=int, default=2_000_000)
    ap.add_argument("--tsize", type=int, default=60_000_000)
    ap.add_argument("--qsize", type=int, default=50_000_000)
    ap.add_argument("--loci", type=int, default=2000)
    ap.add_argument("--seed", type=int, default=None)
    ap.add_argument("--no-ref", action="store_true")
    ap.add_argument("--tmp", default=os.environ.get("TMPDIR", "/tmp"))
    a = ap.parse_args()
    if a.seed is None:
        a.seed = {"scorechain": 42, "chainnet": 42, "c5": 1234}.get(a.tool, 7)
    {"axtchain": axtchain, "cleaner": cleaner, "scorechain": scorechain,
     "chainnet": chainnet, "c5": c5, "microjobs": microjobs}[a.tool](a)


if __name__ == "__main__":
    main()
