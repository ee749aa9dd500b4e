#!/usr/bin/env python3
"""bench.py -- aligned Gbases scored/sec, chainNet -rescore hg38-mm10 (BASELINE.json).

Workload (synthetic, seeded): target = hg38 chr1
(248,956,422 bp), query = all 66 mm10 sequences (2.73 Gb), 2e5 planted
chains (power-law blocks/chain, geometric 40-bp blocks, 12% substitutions,
50% '-' strand, 20% short spurious chains), written as .2bit genomes,
chrom.sizes files and a score-sorted .chain file.

Headline (`value`, SURVEY §8(d) primary metric): ONE STEP = one end-to-end
`bin/chainNet in.chain t.sizes q.sizes t.net q.net -rescore -tNibDir=t.2bit
-qNibDir=q.2bit -linearGap=loose` invocation (the drop-in tool: process
start, chain parse, host netting, 2bit genomes + chains to HBM, GPU
rescoring of every partial target fill, both nets written).  value = the
aligned bases of the netted input chains (score >= 0) / wall time per step.

N > 1 (torchrun, one process per GPU): weak scaling, C2 per GPU.  The input
is ONE chain set over N target chromosomes: N replicas of C2's target
chromosome (chr1, chr1_r1, ..., same sequence) and of its chains (renamed,
ids renumbered, interleaved in score order), against the same mm10 query.
Every step runs the tool on every rank over that input with -nranks=N
-rank=r: rank r nets the chromosome sides it owns (contiguous runs of each
sizes file, balanced by length: one target chromosome per rank, 1/N of the
query chromosomes), parses only the chains on its sides, loads only its
target sequence, rescores its target fills on its own GPU and writes its
part; rank 0 assembles both nets.  No data-path collective (the netting
partitions by chromosome side); torch.distributed (RCCL) carries the
barriers and the max-over-ranks clock.  value = netted aligned bases of the
whole set / wall time.

Also reported:
  kernel   -- the GPU rescoring call alone (gac_score_ranges_device over the
              C2 partial fills, inputs resident in HBM), HIP-event timed;
  roofline -- its dominant kernel k_tile: algorithmic bytes per launch
               / k_tile's average launch time, vs 8 TB/s;
  cpu_baseline -- the reference chainNet compiled from /root/reference
              (oracle/_ref/chainNet, test infrastructure) on the same files on
              this host: one process (the reference is single-threaded) and a
              per-chromosome-side split over all cores; nets compared byte
              for byte with ours.
"""
import argparse
import filecmp
import json
import os
import subprocess
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
BLASTZ = np.array([[91, -114, -31, -123], [-114, 100, -125, -31], [-31, -125, 100, -114],
                   [-123, -31, -114, 91]], np.int32)
METRIC = "aligned Gbases scored/sec, chainNet -rescore hg38-mm10, 1/2/4/8 MI355X"
TOOL = os.path.join(REPO, "genomealignmenttools_amd", "bin", "chainNet")
REF_TOOL = os.path.join(REPO, "oracle", "_ref", "chainNet")


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--chains", type=int, default=200_000)
    p.add_argument("--seed", type=int, default=42)
    p.add_argument("--workload", choices=["chainnet", "rescore", "scorechain"], default="chainnet",
                   help="chainnet: end-to-end bin/chainNet -rescore (headline); rescore / "
                        "scorechain: the GPU scoring call alone as the step")
    p.add_argument("--kernel-steps", type=int, default=20)
    p.add_argument("--no-kernel", action="store_true", help="skip the kernel/roofline leg")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-all-cores", action="store_true",
                   help="skip the reference's per-chromosome-side all-cores run")
    p.add_argument("--prof", choices=["tile", "all", "none"], default="tile",
                   help="kernels bracketed by HIP events in the kernel leg (the roofline "
                        "needs k_tile's)")
    p.add_argument("--order", choices=["chain", "net", "t", "q"], default="net",
                   help="kernel leg: ranges in .net output order (as bin/chainNet submits "
                        "them), (chain, tStart), target start, or (query sequence, forward "
                        "query position) order")
    p.add_argument("--tmp", default=os.environ.get("TMPDIR", "/tmp"))
    p.add_argument("--no-pmc", action="store_true",
                   help="roofline.traffic from the committed profile instead of this run's "
                        "rocprofv3 counter passes")
    p.add_argument("--pmc-child", action="store_true", help=argparse.SUPPRESS)
    p.add_argument("--gen-only", action="store_true", help=argparse.SUPPRESS)
    p.add_argument("--replicas", type=int, default=1, help=argparse.SUPPRESS)
    return p.parse_args()


def host_threads():
    v = os.environ.get("GAC_THREADS") or os.environ.get("OMP_NUM_THREADS")
    return int(v) if v else len(os.sched_getaffinity(0))


# ---------------------------------------------------------------- input files
def c2_files(args):
    """C2 written once per box under --tmp: t.2bit, q.2bit, *.sizes, in.chain."""
    from genomealignmenttools_amd import chainfile, synth
    d = os.path.join(args.tmp, f"gac_bench_c2_{args.chains}_{args.seed}")
    p = lambda x: os.path.join(d, x)
    if not os.path.exists(p("info.json")):
        os.makedirs(d, exist_ok=True)
        t0 = time.time()
        tg, qg, ca = synth.c2_case(seed=args.seed, n_chains=args.chains)
        synth.write_2bit(tg, p("t.2bit"))
        synth.write_2bit(qg, p("q.2bit"))
        synth.write_sizes(tg.sizes, p("t.sizes"))
        synth.write_sizes(qg.sizes, p("q.sizes"))
        chainfile.write_chains(ca, p("in.chain"))
        # the netting loop stops at the first chain below minScore (0 with
        # -rescore, chainNet.c:949-952,1022): those chains' aligned bases
        # are the metric's numerator
        neg = np.nonzero(ca.score < 0)[0]
        stop = int(neg[0]) if len(neg) else ca.n
        info = {"chains": ca.n, "blocks": int(len(ca.blk_size)),
                "input_aligned_bases": ca.aligned_bases(),
                "netted_chains": stop,
                "netted_aligned_bases": int(ca.blk_size[:ca.blk_off[stop]].sum(dtype=np.int64))}
        with open(p("info.json.tmp"), "w") as f:
            json.dump(info, f)
        os.rename(p("info.json.tmp"), p("info.json"))
        log(f"C2: {info} written in {time.time() - t0:.1f}s")
    with open(p("info.json")) as f:
        return d, json.load(f)


def _replicate_2bit(src, dst, names):
    """A version-0 .2bit holding the one sequence of `src` under every name
    (its record bytes copied, the index rebuilt)."""
    import struct
    with open(src, "rb") as f:
        data = f.read()
    magic, _, cnt, _ = struct.unpack_from("<IIII", data, 0)
    assert cnt == 1, src
    nl = data[16]
    rec = data[struct.unpack_from("<I", data, 17 + nl)[0]:]
    off = 16 + sum(1 + len(n) + 4 for n in names)
    with open(dst + ".tmp", "wb") as f:
        f.write(struct.pack("<IIII", magic, 0, len(names), 0))
        for k, n in enumerate(names):
            f.write(struct.pack("<B", len(n)) + n.encode() + struct.pack("<I", off + k * len(rec)))
        for _ in names:
            f.write(rec)
    os.rename(dst + ".tmp", dst)


def _replicate_chains(src, dst, names):
    """Every chain of `src` once per target name (tName replaced), copies
    adjacent (the file stays sorted by score), ids 1..n in file order."""
    with open(src, "rb") as f:
        data = f.read()
    head, sep, body = data.partition(b"chain ")
    out, nid = [head], 0
    enc = [n.encode() for n in names]
    for rec in (sep + body).split(b"\n\n"):
        if not rec.strip():
            continue
        hdr, _, blocks = rec.partition(b"\n")
        w = hdr.split(b" ")
        for nm in enc:
            nid += 1
            w[2] = nm
            w[12:] = [str(nid).encode()]
            out.append(b" ".join(w) + b"\n" + blocks + b"\n\n")
    with open(dst + ".tmp", "wb") as f:
        f.write(b"".join(out))
    os.rename(dst + ".tmp", dst)


def c2n_files(args, n):
    """The N>1 input: C2 replicated per rank (see the module docstring)."""
    d1, info1 = c2_files(args)
    d = d1 + f"_x{n}"
    p = lambda x: os.path.join(d, x)
    if not os.path.exists(p("info.json")):
        os.makedirs(d, exist_ok=True)
        t0 = time.time()
        names = ["chr1"] + [f"chr1_r{k}" for k in range(1, n)]
        tsize = open(os.path.join(d1, "t.sizes")).read().split()[1]
        with open(p("t.sizes"), "w") as f:
            f.write("".join(f"{nm}\t{tsize}\n" for nm in names))
        _replicate_2bit(os.path.join(d1, "t.2bit"), p("t.2bit"), names)
        _replicate_chains(os.path.join(d1, "in.chain"), p("in.chain"), names)
        for x in ("q.2bit", "q.sizes"):
            if not os.path.exists(p(x)):
                os.symlink(os.path.join(d1, x), p(x))
        info = {k: v * n for k, v in info1.items()}
        info["replicas"] = n
        with open(p("info.json.tmp"), "w") as f:
            json.dump(info, f)
        os.rename(p("info.json.tmp"), p("info.json"))
        log(f"C2 x{n}: written in {time.time() - t0:.1f}s")
    with open(p("info.json")) as f:
        return d, json.load(f)


def tool_cmd(d, out, world, rank, extra=()):
    p = lambda x: os.path.join(d, x)
    cmd = [TOOL, p("in.chain"), p("t.sizes"), p("q.sizes"), out + ".t.net", out + ".q.net",
           "-rescore", f"-tNibDir={p('t.2bit')}", f"-qNibDir={p('q.2bit')}", "-linearGap=loose"]
    if world > 1:
        cmd += [f"-nranks={world}", f"-rank={rank}", f"-gpu={int(os.environ.get('LOCAL_RANK', rank))}"]
    return cmd + list(extra)


def run_tool(cmd, outs, env=None):
    for o in outs:  # (a truncated-and-rewritten file may be flushed on close)
        if os.path.exists(o):
            os.remove(o)
    # close_fds=False lets subprocess use posix_spawn (vfork): the launch
    # costs the same whatever this process's size
    r = subprocess.run(cmd, capture_output=True, text=True, env=env, timeout=900, close_fds=False)
    if r.returncode != 0:
        raise RuntimeError(f"{cmd[0]} rc={r.returncode}: {r.stderr[-3000:]}")
    return r


# ---------------------------------------------------------------- kernel leg
def kernel_ranges(args, d):
    """The kernel leg's chain set and ranges (host only, no device): the C2
    partial target fills (or whole chains), in the --order order; cached as
    .npy beside the input for the counter passes' child processes."""
    from genomealignmenttools_amd import chainfile
    from genomealignmenttools_amd.chainnet import net_fills
    from genomealignmenttools_amd.synth import read_sizes
    p = lambda x: os.path.join(d, x)
    ca = chainfile.read_chains(p("in.chain"))
    cache = p(f"ranges.{args.workload}.{args.order}.npy")
    if os.path.exists(cache):
        return ca, np.load(cache)
    if args.workload == "scorechain":
        ranges = np.stack([np.arange(ca.n, dtype=np.int32), ca.tstart, ca.tend], 1)
    else:
        fills = net_fills(ca, read_sizes(p("t.sizes")), read_sizes(p("q.sizes")), min_score=0.0)
        part = fills["partial"]
        ranges = np.stack([fills["chain"][part], fills["start"][part], fills["end"][part]], 1)
    if args.order == "chain":
        ranges = ranges[np.lexsort((ranges[:, 1], ranges[:, 0]))]
    elif args.order == "t":
        ranges = ranges[np.argsort(ranges[:, 1], kind="stable")]
    elif args.order == "q":
        ranges = ranges[np.lexsort(_query_key(ca, ranges)[::-1])]
    ranges = np.ascontiguousarray(ranges, np.int32)
    np.save(cache + ".tmp.npy", ranges)
    os.rename(cache + ".tmp.npy", cache)
    return ca, ranges


def kernel_leg(args, d, steps, ca, ranges, pmc=None):
    """The GPU rescoring call alone (inputs resident in HBM), HIP-event timed:
    the roofline of k_tile and a per-kernel breakdown.  pmc: this run's
    counter-pass traffic (pmc_traffic) or None."""
    from genomealignmenttools_amd._lib import GAC_K_COMBINE, GAC_K_PLAN, GAC_K_TILE
    from genomealignmenttools_amd.gachain import GAC_Q, GAC_T, Engine, GapCosts
    p = lambda x: os.path.join(d, x)
    t0 = time.time()
    e = Engine(int(os.environ.get("LOCAL_RANK", "0")))
    e.load_2bit(GAC_T, p("t.2bit"))
    e.load_2bit(GAC_Q, p("q.2bit"))
    e.set_scoring(BLASTZ, GapCosts("loose"))
    cs = e.upload_chains(ca)
    n = len(ranges)
    d_r = e.dev_alloc(ranges.nbytes)
    e.h2d(d_r, ranges)
    d_g = e.dev_alloc(8 * n)
    d_a = e.dev_alloc(4 * n)
    ali = np.zeros(n, np.int32)
    e.score_ranges_device(cs, d_r, n, d_g, d_a)
    e.synchronize()
    e.d2h(ali, d_a)
    bases = int(ali.sum(dtype=np.int64))
    nblk = _window_blocks(ca, ranges)
    log(f"kernel leg: {n} ranges, {bases} bases, {nblk} window blocks ({time.time() - t0:.1f}s setup)")
    for _ in range(3):
        e.score_ranges_device(cs, d_r, n, d_g, d_a)
    e.synchronize()
    e.prof_reset()
    if args.prof != "none":
        e.prof_enable(True, None if args.prof == "all" else [GAC_K_TILE])
    t0 = time.perf_counter()
    for _ in range(steps):
        e.score_ranges_device(cs, d_r, n, d_g, d_a)
    e.synchronize()
    dt = time.perf_counter() - t0
    e.prof_enable(False)
    tile_ms, tile_n = e.prof_read(GAC_K_TILE)
    e.prof_reset()
    e.prof_enable(True)
    for _ in range(min(steps, 5)):
        e.score_ranges_device(cs, d_r, n, d_g, d_a)
    e.synchronize()
    e.prof_enable(False)
    kern_ms = {name: e.prof_read(k)[0] / max(e.prof_read(k)[1], 1)
               for name, k in (("plan+tilemap", GAC_K_PLAN), ("tile", GAC_K_TILE),
                               ("combine", GAC_K_COMBINE))}
    if args.prof == "none":
        tile_ms, tile_n = kern_ms["tile"], 1
    cs.close()
    e.close()
    # algorithmic bytes per k_tile launch: 0.75 B/base (t+q 2-bit + t+q
    # N-mask bits) + 12 B/window block + 44 B/range
    algo = 0.75 * bases + 12.0 * nblk + 44.0 * n
    tile_s = (tile_ms / 1e3) / max(tile_n, 1)
    achieved = algo / tile_s / 1e9
    kernel = {"workload": ("chainNet -rescore partial target fills" if args.workload != "scorechain"
                           else "scoreChain whole chains, global + local"),
              "value": bases * steps / dt / 1e9, "unit": "Gbases/s", "ms_per_step": dt / steps * 1e3,
              "steps": steps, "ranges": n, "order": args.order, "scored_bases": bases,
              "window_blocks": nblk,
              "kernel_ms": kern_ms}
    roof = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS, "traffic": None,
            "kernel": "k_tile", "kernel_avg_ms": tile_s * 1e3, "algo_bytes_per_launch": algo}
    if pmc and pmc.get("hbm_bytes"):
        roof["traffic"] = pmc["hbm_bytes"]
        roof["traffic_source"] = pmc["source"]
        roof["traffic_over_algo"] = pmc["hbm_bytes"] / algo
        roof["traffic_kernel_avg_ms"] = pmc.get("avg_ms")
    else:
        roof["traffic"] = _pmc_traffic(args, n, nblk)
        if roof["traffic"]:
            roof["traffic_source"] = "committed profile " + os.path.relpath(TRAFFIC_FILE, REPO)
    return kernel, roof


PMC_PASSES = ("TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum",
              "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum")


def pmc_traffic(args):
    """HBM-side bytes per k_tile launch, measured in this run: two rocprofv3
    --kernel-trace --pmc passes (no other trace domains; 3 and 2 TCC counters)
    over a child process that runs the kernel leg's call.  Bytes by request
    size, as MI355X_MICROARCH.md's HBM section prescribes for gfx950 (not
    FETCH_SIZE, which tallies every request at 64 B): reads = 32 n32 + 64 n64
    + 128 n128, writes = 64 n64 + 32 (n - n64).  Run before this process
    touches the GPU.  Returns None on any failure (reported, never fatal)."""
    import csv
    import glob
    import shutil
    import tempfile
    if not shutil.which("rocprofv3"):
        return None
    child = [sys.executable, os.path.abspath(__file__), "--pmc-child", "--chains", str(args.chains),
             "--seed", str(args.seed), "--workload", args.workload, "--order", args.order,
             "--tmp", args.tmp]
    vals, durs = {}, []
    root = tempfile.mkdtemp(prefix="gac_pmc_", dir="/tmp")
    env = dict(os.environ, TMPDIR="/tmp")
    for i, counters in enumerate(PMC_PASSES):
        out = os.path.join(root, f"pass{i}")
        cmd = ["timeout", "-s", "KILL", "180", "rocprofv3", "--kernel-trace", "--pmc",
               *counters.split(), "--output-format", "csv", "-d", out, "-o", "run", "--", *child]
        r = subprocess.run(cmd, capture_output=True, text=True, cwd="/tmp", env=env, timeout=240)
        if r.returncode != 0:
            log(f"pmc pass {i} rc={r.returncode}: {r.stderr[-800:]}")
            return None
        per = {}
        for path in glob.glob(os.path.join(out, "**", "*counter_collection.csv"), recursive=True):
            with open(path) as f:
                for row in csv.DictReader(f):
                    if "k_tile<" not in row["Kernel_Name"]:  # (not k_tilemap*)
                        continue
                    key = (row["Dispatch_Id"], row["Counter_Name"])
                    per[key] = per.get(key, 0.0) + float(row["Counter_Value"])
        by = {}
        for (_, c), v in per.items():
            by.setdefault(c, []).append(v)
        if not by:
            log(f"pmc pass {i}: no k_tile rows")
            return None
        vals.update({c: sum(v) / len(v) for c, v in by.items()})
        for path in glob.glob(os.path.join(out, "**", "*kernel_trace.csv"), recursive=True):
            with open(path) as f:
                for row in csv.DictReader(f):
                    if "k_tile<" in row["Kernel_Name"]:
                        durs.append(int(row["End_Timestamp"]) - int(row["Start_Timestamp"]))
    shutil.rmtree(root, ignore_errors=True)
    try:
        rd = (32.0 * vals["TCC_EA0_RDREQ_32B_sum"] + 64.0 * vals["TCC_EA0_RDREQ_64B_sum"]
              + 128.0 * vals["TCC_EA0_RDREQ_128B_sum"])
        w64 = vals["TCC_EA0_WRREQ_64B_sum"]
        wr = 64.0 * w64 + 32.0 * (vals["TCC_EA0_WRREQ_sum"] - w64)
    except KeyError as ex:
        log(f"pmc: missing counter {ex}")
        return None
    return {"hbm_bytes": rd + wr, "hbm_read_bytes": rd, "hbm_write_bytes": wr,
            "avg_ms": (sum(durs) / len(durs) / 1e6) if durs else None,
            "source": "this run: rocprofv3 --kernel-trace --pmc " + " | ".join(PMC_PASSES)
                      + " (k_tile dispatches, mean)"}


def pmc_child(args):
    """The counter passes' workload: the kernel leg's call, a few times."""
    d, _ = c2_files(args)
    ca, ranges = kernel_ranges(args, d)
    kernel_leg(args, d, 3, ca, ranges)


TRAFFIC_FILE = os.path.join(REPO, "profiles", "k_tile_traffic.json")


def _pmc_traffic(args, n, nblk):
    """HBM bytes per k_tile launch from the committed PMC profile of this same
    kernel-leg workload (scripts/gpu_counters.sh + scripts/pmc_summary.py),
    or None when no profile matches it."""
    try:
        with open(TRAFFIC_FILE) as f:
            t = json.load(f)
    except (OSError, ValueError):
        return None
    wl = "scorechain" if args.workload == "scorechain" else "rescore"
    if (t.get("workload") != wl or t.get("ranges") != n or t.get("blocks") != nblk
            or t.get("chains") != args.chains or t.get("seed") != args.seed
            or t.get("order", "net") != args.order):
        return None
    return t.get("hbm_bytes_per_launch")


def _query_key(ca, ranges):
    """(query sequence id, forward-strand query position of the first window
    block) per range: the query-plane order of the fills."""
    names = {n: i for i, n in enumerate(dict.fromkeys(ca.qname))}
    qid = np.array([names[n] for n in ca.qname], np.int64)[ranges[:, 0]]
    pos = np.zeros(len(ranges), np.int64)
    for i, (c, s, _) in enumerate(ranges):
        a, b = int(ca.blk_off[c]), int(ca.blk_off[c + 1])
        k = a + int(np.searchsorted(ca.blk_t[a:b] + ca.blk_size[a:b], s, side="right"))
        k = min(k, b - 1)
        q = int(ca.blk_q[k])
        pos[i] = int(ca.qsize[c]) - q if ca.qstrand[c] else q
    return qid, pos


def _window_blocks(ca, ranges):
    """Blocks selected by each range (host binary search, for the byte model)."""
    tot = 0
    for c, s, e in ranges:
        bt, _, bs = ca.blocks(int(c))
        if s <= bt[0] and e >= bt[-1] + bs[-1]:
            tot += len(bt)
            continue
        lo = np.searchsorted(bt + bs, s, side="right")
        hi = np.searchsorted(bt, e, side="left")
        tot += max(0, int(hi - lo))
    return tot


# ---------------------------------------------------------------- CPU baseline
def cpu_baseline(args, d, info, ours):
    """The reference chainNet (oracle/_ref, compiled from /root/reference) on
    the same files: one process, then split per chromosome side over all
    host cores; nets compared with ours."""
    p = lambda x: os.path.join(d, x)
    if not os.path.exists(REF_TOOL):
        return {"error": f"{REF_TOOL} not built (make ref)"}
    opts = ["-rescore", f"-tNibDir={p('t.2bit')}", f"-qNibDir={p('q.2bit')}", "-linearGap=loose"]
    ref = p("ref")
    t0 = time.time()
    run_tool([REF_TOOL, p("in.chain"), p("t.sizes"), p("q.sizes"), ref + ".t.net", ref + ".q.net"]
             + opts, [ref + ".t.net", ref + ".q.net"])
    t1 = time.time() - t0
    same = (filecmp.cmp(ours + ".t.net", ref + ".t.net", False)
            and filecmp.cmp(ours + ".q.net", ref + ".q.net", False))
    log(f"cpu baseline: reference chainNet -rescore {t1:.2f}s, nets identical: {same}")
    out = {"value": info["netted_aligned_bases"] / t1 / 1e9, "unit": "Gbases/s", "cores": 1,
           "kind": "reference", "seconds": t1, "identical_nets": same,
           "sample": f"the whole workload: reference chainNet -rescore (oracle/_ref) on the same "
                     f"C2 files, one process ({t1:.2f}s)"}
    if not args.no_all_cores:
        try:
            out["all_cores"] = ref_all_cores(d, opts, ref)
        except Exception as ex:  # reported, never fatal
            out["all_cores"] = {"error": str(ex)[:300]}
    return out


def ref_all_cores(d, opts, ref):
    """The reference run per chromosome side over all host cores: a target
    sequence's net depends only on the chains on it (a query sequence's
    likewise), so the chains are split by target sequence (target nets) and
    by query sequence (query nets) and the reference runs on every group
    concurrently; the groups' nets are reassembled and compared."""
    from concurrent.futures import ThreadPoolExecutor
    p = lambda x: os.path.join(d, x)
    gd = p("ref_groups")
    os.makedirs(gd, exist_ok=True)
    groups = _split_chain_file(p("in.chain"), gd)
    cores = host_threads()
    jobs = []
    for side, name, path in groups:
        o = os.path.join(gd, f"{side}.{len(jobs)}")
        jobs.append((side, name, [REF_TOOL, path, p("t.sizes"), p("q.sizes"), o + ".t.net",
                                  o + ".q.net"] + opts, o))
    t0 = time.time()
    with ThreadPoolExecutor(max_workers=cores) as ex:
        list(ex.map(lambda j: run_tool(j[2], [j[3] + ".t.net", j[3] + ".q.net"]), jobs))
    wall = time.time() - t0
    same = True
    for side in ("t", "q"):
        parts = {}
        for s, name, _, o in jobs:
            if s == side:
                with open(o + f".{side}.net") as f:
                    parts[name] = _net_sections(f.read())[1].get(name, "")
        with open(ref + f".{side}.net") as f:
            whole = f.read()
        meta, _, order = _net_sections(whole)
        same = same and meta + "".join(parts.get(k, "") for k in order) == whole
    import shutil
    shutil.rmtree(gd, ignore_errors=True)
    log(f"cpu baseline (all cores): {len(jobs)} reference runs on {cores} cores, {wall:.2f}s, "
        f"reassembled nets identical: {same}")
    return {"seconds": wall, "cores": cores, "processes": len(jobs), "identical_nets": same}


def _split_chain_file(path, gd):
    """Chain text split by target and by query sequence (file order kept,
    leading '#' lines copied to every group) -> [(side, sequence, file)]."""
    meta, tg, qg = [], {}, {}
    cur, cur_t, cur_q = [], None, None

    def flush():
        if cur_t is not None:
            rec = "\n".join(cur) + "\n"
            tg.setdefault(cur_t, []).append(rec)
            qg.setdefault(cur_q, []).append(rec)
    with open(path) as f:
        for line in f.read().split("\n"):
            if cur_t is None and line.startswith("#"):
                meta.append(line + "\n")
            elif line.startswith("chain "):
                flush()
                w = line.split()
                cur, cur_t, cur_q = [line], w[2], w[7]
            elif cur_t is not None:
                cur.append(line)
    flush()
    out = []
    for side, g in (("t", tg), ("q", qg)):
        for k, (name, recs) in enumerate(g.items()):
            fn = os.path.join(gd, f"in.{side}{k}.chain")
            with open(fn, "w") as f:
                f.write("".join(meta) + "".join(recs))
            out.append((side, name, fn))
    return out


def _net_sections(text):
    """('#' header, {sequence: its 'net' section}, sequence order) of .net text."""
    meta_end = 0
    while text.startswith("#", meta_end):
        meta_end = text.index("\n", meta_end) + 1
    secs, order = {}, []
    pos = meta_end
    while pos < len(text):
        nxt = text.find("\nnet ", pos)
        end = len(text) if nxt < 0 else nxt + 1
        name = text[pos:text.index("\n", pos)].split()[1]
        secs[name] = text[pos:end]
        order.append(name)
        pos = end
    return text[:meta_end], secs, order


# ---------------------------------------------------------------- main
def main():
    args = parse()
    if args.gen_only:
        c2_files(args)
        if args.replicas > 1:
            c2n_files(args, args.replicas)
        return
    if args.pmc_child:
        pmc_child(args)
        return
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if os.environ.get("GAC_BENCH_ONE_GPU"):  # rehearsal on a one-GPU box: every rank on device 0
        local = 0
        os.environ["LOCAL_RANK"] = "0"
    if world > 1:
        import torch
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        if os.environ.get("GAC_BENCH_ONE_GPU"):  # (RCCL wants one device per rank)
            dist.init_process_group("gloo", rank=rank, world_size=world)
        else:
            dist.init_process_group("nccl", rank=rank, world_size=world,
                                    device_id=torch.device(f"cuda:{local}"))

    def barrier():
        if dist is not None:
            dist.barrier()

    files = (lambda: c2_files(args)) if world == 1 else (lambda: c2n_files(args, world))
    if rank == 0:  # generated in a child process: this one stays small
        subprocess.run([sys.executable, os.path.abspath(__file__), "--gen-only", "--chains",
                        str(args.chains), "--seed", str(args.seed), "--tmp", args.tmp,
                        "--replicas", str(world)], check=True)
        d, info = files()
    barrier()
    if rank != 0:
        d, info = files()  # written by rank 0 (same node)
    out_base = os.path.join(d, f"ours.r{world}")
    outs = [out_base + ".t.net", out_base + ".q.net"]
    cmd = tool_cmd(d, out_base, world, rank)

    # every rank of one step shares a marker token (tells this step's part
    # markers from an earlier, failed one's; see gt_ranks_place)
    run_id = f"{os.environ.get('TORCHELASTIC_RUN_ID', 'x')}-{os.environ.get('MASTER_PORT', '0')}"
    step_no = [0]

    def step_env():
        step_no[0] += 1
        return dict(os.environ, GAC_RANK_TOKEN=f"{run_id}-{step_no[0]}")

    if args.workload == "chainnet":
        for _ in range(args.warmup):
            barrier()
            run_tool(cmd, outs if rank == 0 else [], env=step_env())
        barrier()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            run_tool(cmd, outs if rank == 0 else [], env=step_env())
            barrier()  # rank 0 finishes last (it waits for every part)
        dt = time.perf_counter() - t0
        if dist is not None:
            from genomealignmenttools_amd.shard import reduce_time_and_work
            dev = "cpu" if os.environ.get("GAC_BENCH_ONE_GPU") else f"cuda:{local}"
            dt, _ = reduce_time_and_work(dist, dt, 0.0, device=dev)
        step_s = dt / args.steps
        stages = None
        if world == 1:  # one more, untimed run for the per-stage breakdown
            r = run_tool(cmd + ["-verbose=2"], outs)
            stages = [line.strip() for line in r.stderr.splitlines() if "[stage]" in line]
        out = {
            "metric": METRIC,
            "value": info["netted_aligned_bases"] / step_s / 1e9,
            "unit": "Gbases/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": step_s * 1e3, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "int64",
            "data": "synthetic (seeded C2: hg38 chr1 x mm10 sizes, planted chains; no real genomes)"
                    + ("" if world == 1 else f"; C2 replicated x{world}: {world} target "
                       "chromosomes (copies of C2's chr1) in one chain set"),
            "config": {"workload": "chainNet -rescore end to end (bin/chainNet, C2"
                                   + (")" if world == 1 else f" per GPU, one set over {world} "
                                      "target chromosomes, chromosome sides split across ranks)"),
                       **info, "parallelism": f"chromosome-side shards x{world}",
                       "host_threads_per_rank": host_threads(), "tool_stages": stages},
        }
    else:
        out = {"metric": METRIC, "n_gpus": world, "unit": "Gbases/s", "higher_is_better": True,
               "scaling": "weak", "vs_baseline": None, "dtype": "int64",
               "data": "synthetic (seeded C2)", "config": {"workload": args.workload, **info}}
    if rank == 0 and not args.no_kernel:
        ca, ranges = kernel_ranges(args, d)
        # counter passes in child processes before this one opens the device
        pmc = None if (args.no_pmc or world > 1) else pmc_traffic(args)
        kernel, roof = kernel_leg(args, d, args.kernel_steps, ca, ranges, pmc)
        out["kernel"] = kernel
        out["roofline"] = roof
        if args.workload != "chainnet":  # the kernel call itself is the step
            out.update(value=kernel["value"], steps=args.kernel_steps, warmup=3,
                       ms_per_step=kernel["ms_per_step"])
    if rank == 0 and world == 1 and not args.no_cpu_baseline and args.workload == "chainnet":
        try:
            out["cpu_baseline"] = cpu_baseline(args, d, info, out_base)
        except Exception as ex:  # reported, never fatal
            out["cpu_baseline"] = {"error": str(ex)[:300]}
    if rank == 0:
        print(json.dumps(out), flush=True)
    barrier()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
