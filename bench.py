#!/usr/bin/env python3
"""bench.py -- aligned Gbases scored/sec, chainNet -rescore hg38-mm10, 1/2/4/8 MI355X
(BASELINE.json).

Headline workload (synthetic, seeded): the whole
genome -- all 455 hg38 sequences as target x all 66 mm10 sequences as query,
5e6 chains (C2's chain model: power-law blocks/chain, geometric 40-bp
blocks, 70/28/2 % gap mixture, 12 % substitutions, 50 % '-' strand, 20 %
short spurious chains; chains per target sequence in proportion to its
length), written as .2bit genomes, chrom.sizes files and a score-sorted
.chain file by the C generator gac_synth (bench infrastructure,
csrc/synth/gac_synth.c).

ONE STEP = one end-to-end `bin/chainNet in.chain t.sizes q.sizes t.net q.net
-rescore -tNibDir=t.2bit -qNibDir=q.2bit -linearGap=loose` over that input:
process start, chain parse, host netting, 2bit genomes + chains to HBM, GPU
rescoring of every partial target fill, both nets written, process exit.
value = the aligned bases of the netted input chains (score >= 0) / wall time
per step (SURVEY §8(d) primary metric).

N > 1 (one process per GPU): `python bench.py --gpus N` starts the N ranks
itself (one torch.distributed.run child, before anything touches a GPU) unless
it already runs under torchrun; every rank checks that the process group
(backend nccl = RCCL) has --gpus ranks, and n_gpus is that group's size.
STRONG scaling on the same fixed input.
Every rank runs the tool with -nranks=N -rank=r -gpu=LOCAL_RANK each step:
rank r nets the chromosome sides it owns (contiguous runs of each sizes file,
balanced by length), parses only the chains on its sides, loads only its
target sequences, rescores its target fills on its GPU and writes its part of
both nets in place.  The netting partitions by chromosome side, so there is no
data-path collective; torch.distributed (RCCL) carries the barriers and the
max-over-ranks clock.  value = the set's netted aligned bases / step time.

Also reported (rank 0):
  c2          -- configs[1]: the same tool on C2 (hg38 chr1 x mm10, 2e5
                 chains), N = 1 only, with its reference time;
  kernel      -- the GPU rescoring call alone (gac_score_ranges_device over
                 exactly the partial fills the tool rescored in the headline,
                 dumped by GAC_DUMP_RANGES), inputs resident in HBM, HIP-event
                 timed on the launch stream;
  roofline    -- its dominant kernel k_tile against the SURVEY §8(d) RANGE
                 model: 32 B/range + 8 B/window block + 0.75 B/scored base;
                 traffic = HBM-side bytes from rocprofv3 counter passes in this
                 run (N = 1);
  scorechain  -- the whole-chain scoring call (global + local, the scoreChain
                 path) over every C5 chain, with its own roofline on the
                 §8(d) full-chain model: 0.75 B/base + 12 B/block + 44 B/chain;
  cpu_baseline -- the reference chainNet compiled from /root/reference
                 (oracle/_ref/chainNet, test infrastructure) timed on this
                 host, one process (it is single-threaded), on a bounded
                 sample of the same workload: the C5 chains on chr21 + chr22
                 (their target nets are compared with ours byte for byte).
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
PKG = os.path.join(REPO, "genomealignmenttools_amd")
TOOL = os.path.join(PKG, "bin", "chainNet")
SYNTH = os.path.join(PKG, "libexec", "gac_synth")
REF_TOOL = os.path.join(REPO, "oracle", "_ref", "chainNet")
SC_TOOL = os.path.join(PKG, "bin", "scoreChain")
AXT_TOOL = os.path.join(PKG, "bin", "axtChain")
REF_SC_TOOL = os.path.join(REPO, "oracle", "_ref", "scoreChain")
REF_AXT_TOOL = os.path.join(REPO, "oracle", "_ref", "axtChain")
SAMPLE_TARGETS = ("chr21", "chr22")
# all-cores baseline: the reference split by target chromosome, one process
# per sequence, run side by side (how the reference is parallelised on a
# cluster: chainNet per target chromosome)
ALL_CORES_TARGETS = tuple(f"chr{i}" for i in range(7, 23))


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=5)
    p.add_argument("--warmup", type=int, default=1)
    p.add_argument("--chains", type=int, default=5_000_000, help="C5 chain count")
    p.add_argument("--seed", type=int, default=1234)
    p.add_argument("--c2-chains", type=int, default=200_000)
    p.add_argument("--c2-steps", type=int, default=10)
    p.add_argument("--kernel-steps", type=int, default=20)
    p.add_argument("--no-c2", action="store_true")
    p.add_argument("--no-c3", action="store_true", help="skip the chainCleaner C3 leg")
    p.add_argument("--c3-steps", type=int, default=3)
    p.add_argument("--no-c4", action="store_true", help="skip the axtChain C4 leg")
    p.add_argument("--c4-blocks", type=int, default=50_000_000)
    p.add_argument("--c4-steps", type=int, default=1)
    p.add_argument("--no-c4-ref", action="store_true",
                   help="skip the reference axtChain timed on a C4 pair subset")
    p.add_argument("--no-kernel", action="store_true", help="skip the kernel/roofline legs")
    p.add_argument("--no-scorechain", action="store_true")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-pmc", action="store_true")
    p.add_argument("--tmp", default=os.environ.get("TMPDIR", "/tmp"))
    p.add_argument("--sharded-scorechain", action="store_true",
                   help="N = 1: also run the N > 1 scorechain leg (world-1 RCCL group)")
    p.add_argument("--pmc-child", choices=["fills", "scorechain"], help=argparse.SUPPRESS)
    p.add_argument("--gen-only", action="store_true", help=argparse.SUPPRESS)
    p.add_argument("--launch-check", action="store_true",
                   help="start the ranks, report the process group each one sees, exit")
    return p.parse_args()


# ---------------------------------------------------------------- launching
def free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_cmd(gpus, argv, port):
    """The one child that runs N ranks when `bench.py --gpus N` is started
    without a torchrun environment: torch.distributed.run, one process per
    GPU on this node, rendezvous on 127.0.0.1."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
            f"--nproc-per-node={gpus}", "--master-addr=127.0.0.1", f"--master-port={port}",
            os.path.abspath(__file__), *argv]


def maybe_self_launch(args):
    """`python bench.py --gpus N`, N > 1, outside torchrun: start the N ranks
    as a child process (before anything here touches a GPU) and leave with its
    exit status.  Inside torchrun (WORLD_SIZE set) nothing happens here; the
    ranks check WORLD_SIZE == --gpus themselves."""
    if "WORLD_SIZE" in os.environ or args.gpus <= 1:
        return
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC (RCCL between processes)
    log(f"bench: starting {args.gpus} ranks (torch.distributed.run)")
    r = subprocess.run(launch_cmd(args.gpus, sys.argv[1:], free_port()), env=env)
    sys.exit(r.returncode)


def init_ranks(args):
    """(dist or None, world, rank, local, one_gpu, group): this rank's place.
    One process per GPU: backend nccl (RCCL over xGMI) on cuda:LOCAL_RANK;
    GAC_BENCH_ONE_GPU=1 is the rehearsal with every rank on device 0 over
    gloo.  Fails loudly when the group is not the --gpus the run asked for."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    one_gpu = bool(os.environ.get("GAC_BENCH_ONE_GPU"))
    if one_gpu:
        local = 0
        os.environ["LOCAL_RANK"] = "0"
    if world != args.gpus:
        raise SystemExit(f"bench: --gpus {args.gpus} but WORLD_SIZE={world}")
    if world == 1:
        return None, 1, 0, 0, one_gpu, None
    import torch
    import torch.distributed as dist
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    if one_gpu:  # (RCCL wants one device per rank)
        dist.init_process_group("gloo", rank=rank, world_size=world)
    else:
        ndev = torch.cuda.device_count()
        if ndev < int(os.environ.get("LOCAL_WORLD_SIZE", world)):
            raise SystemExit(f"bench: {ndev} GPUs visible for {world} ranks on this node")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", rank=rank, world_size=world,
                                device_id=torch.device(f"cuda:{local}"))
    if dist.get_world_size() != args.gpus:
        raise SystemExit(f"bench: process group has {dist.get_world_size()} ranks, "
                         f"--gpus {args.gpus}")
    me = {"rank": rank, "local_rank": local, "device": "cpu (rehearsal)" if one_gpu else
          f"cuda:{local}", "pid": os.getpid()}
    if not one_gpu:
        pr = torch.cuda.get_device_properties(local)
        me.update(name=pr.name, uuid=str(getattr(pr, "uuid", "")),
                  pci_bus_id=getattr(pr, "pci_bus_id", None))
    group = [None] * world
    dist.all_gather_object(group, me)
    return dist, world, rank, local, one_gpu, {"backend": dist.get_backend(),
                                               "world_size": dist.get_world_size(),
                                               "ranks": group}


def host_threads():
    v = os.environ.get("GAC_THREADS") or os.environ.get("OMP_NUM_THREADS")
    return int(v) if v else usable_cpus()


def usable_cpus(cpu_max="/sys/fs/cgroup/cpu.max"):
    """The CPUs this process may use: its affinity mask narrowed by its
    cgroup's CPU quota (gac_host_cpus in csrc/host/gac_host.c, the same rule)."""
    n = len(os.sched_getaffinity(0))
    try:
        with open(cpu_max) as f:
            q, per = f.read().split()[:2]
        if q != "max" and int(q) > 0 and int(per) > 0:
            n = min(n, -(-int(q) // int(per)))
    except (OSError, ValueError):
        pass
    return max(1, n)


def rank_tool_threads(world, env, cpus):
    """GAC_THREADS for the tool each of `world` ranks runs (N > 1): the
    caller's GAC_THREADS / OMP_NUM_THREADS wins, except torch.distributed.run's
    own default OMP_NUM_THREADS=1 (it sets it for every worker when the
    launching environment has none; TORCHELASTIC_RUN_ID marks its workers),
    which would run each rank's netting and parsing on one thread.  Else the
    usable CPUs shared by the node's ranks: N ranks x all cores would
    oversubscribe the host.  {} = leave the environment as it is."""
    if world <= 1 or env.get("GAC_THREADS"):
        return {}
    omp = env.get("OMP_NUM_THREADS")
    if omp and not (omp == "1" and env.get("TORCHELASTIC_RUN_ID")):
        return {}
    local_world = int(env.get("LOCAL_WORLD_SIZE", world))
    return {"GAC_THREADS": str(max(1, cpus // local_world))}


def host_cpu():
    """The host the CPU baseline ran on: CPU model, the machine's logical
    CPUs (nproc) and the CPUs this process may use (its share of the box)."""
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {"cpu_model": model, "host_nproc": os.cpu_count(),
            "affinity_cpus": len(os.sched_getaffinity(0))}


# ---------------------------------------------------------------- input files
def c5_files(args):
    """C5 written once per box under --tmp by gac_synth (~15 s on 16 threads)."""
    d = os.path.join(args.tmp, f"gac_bench_c5_{args.chains}_{args.seed}")
    if not os.path.exists(os.path.join(d, "info.json")):
        if not os.path.exists(SYNTH):
            raise SystemExit(f"{SYNTH} missing: run `make synth` (or __graft_entry__.build())")
        t0 = time.time()
        subprocess.run([SYNTH, "c5", d, f"-seed={args.seed}", f"-chains={args.chains}",
                        f"-sizesDir={os.path.join(PKG, 'data')}",
                        f"-threads={min(host_threads(), 32)}"], check=True)
        log(f"C5: written in {time.time() - t0:.1f}s")
    with open(os.path.join(d, "info.json")) as f:
        return d, json.load(f)


def c2_files(args):
    """C2 written once per box under --tmp: t.2bit, q.2bit, *.sizes, in.chain."""
    from genomealignmenttools_amd import chainfile, synth
    d = os.path.join(args.tmp, f"gac_bench_c2_{args.c2_chains}_42")
    p = lambda x: os.path.join(d, x)
    if not os.path.exists(p("info.json")):
        os.makedirs(d, exist_ok=True)
        t0 = time.time()
        tg, qg, ca = synth.c2_case(seed=42, n_chains=args.c2_chains)
        synth.write_2bit(tg, p("t.2bit"))
        synth.write_2bit(qg, p("q.2bit"))
        synth.write_sizes(tg.sizes, p("t.sizes"))
        synth.write_sizes(qg.sizes, p("q.sizes"))
        chainfile.write_chains_fast(ca, p("in.chain"))
        neg = np.nonzero(ca.score < 0)[0]
        stop = int(neg[0]) if len(neg) else ca.n
        info = {"chains": ca.n, "blocks": int(len(ca.blk_size)),
                "input_aligned_bases": ca.aligned_bases(), "netted_chains": stop,
                "netted_aligned_bases": int(ca.blk_size[:ca.blk_off[stop]].sum(dtype=np.int64))}
        with open(p("info.json.tmp"), "w") as f:
            json.dump(info, f)
        os.rename(p("info.json.tmp"), p("info.json"))
        log(f"C2: {info} written in {time.time() - t0:.1f}s")
    with open(p("info.json")) as f:
        return d, json.load(f)


def load_chains_bin(d):
    """chains.bin of gac_synth (layout in csrc/synth/gac_synth.c) -> arrays."""
    path = os.path.join(d, "chains.bin")
    with open(path, "rb") as f:
        assert f.read(8) == b"GACSYN01", path
        n, nb = (int(x) for x in np.fromfile(f, np.int64, 2))
        out = {"n": n, "nb": nb, "score": np.fromfile(f, np.float64, n)}
        for k in ("tseq", "qseq", "tstart", "tend", "qstart", "qend"):
            out[k] = np.fromfile(f, np.int32, n)
        out["strand"] = np.fromfile(f, np.uint8, (n + 7) // 8 * 8)[:n]
        out["off"] = np.fromfile(f, np.int64, n + 1)
        for k in ("bt", "bq", "bs"):
            out[k] = np.fromfile(f, np.int32, nb)
    return out


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


def staged_run(d, out):
    """One untimed single-process run with the stage laps (-verbose=2) and
    the rescored fills dumped for the kernel leg.  Returns the stage lines
    plus the attribution of the parent's wall time: spawn -> the tool's
    process start (fork + exec of the launcher), the tool's own laps (process
    start -> main -> ... -> its exit call), and its exit call -> the parent's
    wait returning (process teardown: HIP runtime / driver)."""
    env = dict(os.environ, GAC_DUMP_RANGES=os.path.join(d, "fills.bin"))
    for o in (out + ".t.net", out + ".q.net"):
        if os.path.exists(o):
            os.remove(o)
    t0 = time.time()
    r = run_tool(tool_cmd(d, out, 1, 0, ["-verbose=2"]), [], env=env)
    t1 = time.time()
    lines = [line.strip() for line in r.stderr.splitlines() if "[stage]" in line]
    clk = {}
    for line in r.stderr.splitlines():
        if line.startswith("[stage-clock]"):
            w = line.split()
            for k in range(1, len(w) - 1, 2):
                clk[w[k]] = float(w[k + 1])
    if {"main", "process-start", "exit"} <= clk.keys():
        lines.append(f"[wall] spawn -> process start {clk['process-start'] - t0:.3f} s, process "
                     f"start -> exit call {clk['exit'] - clk['process-start']:.3f} s, exit call -> "
                     f"parent's wait returns {t1 - clk['exit']:.3f} s (total {t1 - t0:.3f} s)")
    return lines


# ---------------------------------------------------------------- kernel legs
def _window_blocks(ch, ranges):
    """Blocks each range selects (tEnd > s and tStart < e; the whole chain
    when the range covers it), vectorised with a (chain, t) key that is
    monotone over the concatenated block arrays."""
    c = ranges[:, 0].astype(np.int64)
    s, e = ranges[:, 1].astype(np.int64), ranges[:, 2].astype(np.int64)
    nbk = np.diff(ch["off"])
    cid = np.repeat(np.arange(ch["n"], dtype=np.int64), nbk) << 32
    bt = ch["bt"].astype(np.int64)
    lo = np.searchsorted(cid + bt + ch["bs"], (c << 32) + s, side="right")
    hi = np.searchsorted(cid + bt, (c << 32) + e, side="left")
    w = np.maximum(0, hi - lo)
    full = (s <= ch["tstart"][c]) & (e >= ch["tend"][c])
    w[full] = nbk[c[full]]
    return int(w.sum())


class Legs:
    """One device context with C5's genomes and chain set resident in HBM."""

    def __init__(self, d, ch):
        from genomealignmenttools_amd.gachain import GAC_Q, GAC_T, Engine, GapCosts
        t0 = time.time()
        self.e = e = Engine(int(os.environ.get("LOCAL_RANK", "0")))
        e.load_2bit(GAC_T, os.path.join(d, "t.2bit"))
        e.load_2bit(GAC_Q, os.path.join(d, "q.2bit"))
        e.set_scoring(BLASTZ, GapCosts("loose"))
        names = lambda side, path: [ln.split()[0] for ln in open(path) if ln.strip()]
        tmap = np.array([e.seq_index(GAC_T, x) for x in names(GAC_T, os.path.join(d, "t.sizes"))],
                        np.int32)
        qmap = np.array([e.seq_index(GAC_Q, x) for x in names(GAC_Q, os.path.join(d, "q.sizes"))],
                        np.int32)
        self.cs = e.upload_chain_arrays(tmap[ch["tseq"]], qmap[ch["qseq"]], ch["strand"], ch["off"],
                                        ch["bt"], ch["bq"], ch["bs"])
        log(f"legs: genomes + {ch['n']} chains in HBM ({time.time() - t0:.1f}s)")

    def run(self, ranges, want_local, steps):
        """HIP-event timed calls over `ranges` (device-resident; None = every
        chain whole, gac_score_chains_device): the call's wall time per step,
        k_tile's average launch, a per-kernel breakdown and the scored
        bases."""
        from genomealignmenttools_amd._lib import GAC_K_COMBINE, GAC_K_PLAN, GAC_K_TILE
        e, cs = self.e, self.cs
        n = cs.n_chains if ranges is None else len(ranges)
        wins = ranges is not None and ranges.shape[1] == 5  # gac_window records
        d_r = e.dev_alloc(16 if ranges is None else max(ranges.nbytes, 16))
        if ranges is not None:
            e.h2d(d_r, np.ascontiguousarray(ranges, np.int32))
        d_g = e.dev_alloc(8 * n + 8)
        d_l = e.dev_alloc(8 * n + 8) if want_local else 0
        d_a = e.dev_alloc(4 * n + 8)
        if ranges is None:
            call = lambda: e.score_chains_device(cs, d_g, d_a, d_l, want_local)
        elif wins:
            call = lambda: e.score_windows_device(cs, d_r, n, d_g, d_a, d_l, want_local)
        else:
            call = lambda: e.score_ranges_device(cs, d_r, n, d_g, d_a, d_l, want_local)
        for _ in range(3):
            call()
        e.synchronize()
        ali = np.zeros(n, np.int32)
        e.d2h(ali, d_a)
        e.prof_reset()
        e.prof_enable(True, [GAC_K_TILE])
        t0 = time.perf_counter()
        for _ in range(steps):
            call()
        e.synchronize()
        dt = time.perf_counter() - t0
        e.prof_enable(False)
        tile_ms, tile_n = e.prof_read(GAC_K_TILE)
        e.prof_reset()
        e.prof_enable(True)
        for _ in range(min(steps, 5)):
            call()
        e.synchronize()
        e.prof_enable(False)
        kern = {}
        for name, k in (("plan+tilemap", GAC_K_PLAN), ("tile", GAC_K_TILE), ("combine", GAC_K_COMBINE)):
            ms, cnt = e.prof_read(k)
            kern[name] = ms / max(cnt, 1)
        for p in (d_r, d_g, d_a) + ((d_l,) if d_l else ()):
            e.dev_free(p)
        return {"step_ms": dt / steps * 1e3, "tile_ms": tile_ms / max(tile_n, 1), "kernel_ms": kern,
                "bases": int(ali.sum(dtype=np.int64)), "steps": steps}

    def score_all(self):
        """Every chain's (global, local, ali), one untimed call (the check of
        the sharded N > 1 leg)."""
        return self.e.score_chains(self.cs, want_local=True)

    def close(self):
        self.cs.close()
        self.e.close()


def fills_windows(d):
    """The fills the headline rescored, as the tool dumped them
    (GAC_DUMP_RANGES): gac_window records (chain, tStart, tEnd, first block,
    block count)."""
    r = np.fromfile(os.path.join(d, "fills.bin"), np.int32).reshape(-1, 5)
    return np.ascontiguousarray(r)


def roofline(algo, t_ms, pmc, kernel):
    roof = {"bound": "hbm", "achieved": algo / (t_ms / 1e3) / 1e9, "peak": HBM_PEAK_GBS,
            "unit": "GB/s", "traffic": None, "kernel": kernel, "kernel_avg_ms": t_ms,
            "algo_bytes_per_launch": algo}
    roof["frac"] = roof["achieved"] / HBM_PEAK_GBS
    if pmc and pmc.get("hbm_bytes"):
        roof.update(traffic=pmc["hbm_bytes"], traffic_source=pmc["source"],
                    traffic_over_algo=pmc["hbm_bytes"] / algo, traffic_kernel_avg_ms=pmc.get("avg_ms"))
    return roof


GATHER = os.path.join(PKG, "libexec", "gac_gather_ceiling")


def gather_ceiling():
    """The random-128-B-line gather ceiling of this GPU
    (scripts/probes/gather_ceiling.hip): the best line rate over isolated
    16-B loads to random lines of a 2 GiB buffer (k_tile's access shape),
    several loads in flight and occupancies.  None when unavailable."""
    if not os.path.exists(GATHER):
        return None
    try:
        r = subprocess.run(["timeout", "-k", "10", "120", GATHER, "2048"], capture_output=True,
                           text=True, timeout=150)
        line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
        return json.loads(line[-1]) if r.returncode == 0 and line else None
    except (OSError, ValueError, subprocess.SubprocessError):
        return None


def add_ceiling(roof, ceil):
    """frac_of_gather_ceiling: k_tile's measured HBM bytes per second (the
    in-run PMC traffic over its average launch) against the random-line
    gather ceiling measured on the same GPU in the same run."""
    if not roof or not ceil or not ceil.get("ceiling_isolated_GBps"):
        return
    c = ceil["ceiling_isolated_GBps"]
    roof["gather_ceiling"] = {"GBps": c, "shape": ceil.get("ceiling_shape"),
                              "source": "genomealignmenttools_amd/libexec/gac_gather_ceiling "
                                        "(scripts/probes/gather_ceiling.hip), this run"}
    if roof.get("traffic"):
        ms = roof.get("traffic_kernel_avg_ms") or roof["kernel_avg_ms"]
        rate = roof["traffic"] / (ms / 1e3) / 1e9
        roof["traffic_GBps"] = rate
        roof["frac_of_gather_ceiling"] = rate / c


def fills_leg(legs, d, ch, steps, pmc):
    """The headline's rescoring call on its own: gac_score_windows_device over
    the fills with the windows the netting found (what bin/chainNet calls),
    and, for comparison, gac_score_ranges_device over the same (chain, tStart,
    tEnd) ranges (the device searches every window: k_plan)."""
    wins = fills_windows(d)
    res = legs.run(wins, False, steps)
    res_r = legs.run(np.ascontiguousarray(wins[:, :3]), False, steps)
    nblk = _window_blocks(ch, wins[:, :3])
    n = len(wins)
    # SURVEY §8(d) range model: 32 B/range (16 in, 16 out) + 8 B/window block
    # + 0.75 B/scored base (t+q 2-bit + t+q N-mask bits)
    algo = 32.0 * n + 8.0 * nblk + 0.75 * res["bases"]
    kernel = {"workload": "chainNet -rescore: the C5 partial target fills the headline rescored "
                          "(gac_score_windows_device: windows from the netting)",
              "value": res["bases"] / (res["step_ms"] / 1e3) / 1e9, "unit": "Gbases/s",
              "ms_per_step": res["step_ms"], "steps": steps, "ranges": n, "order": "net",
              "scored_bases": res["bases"], "window_blocks": nblk,
              "window_blocks_given": int(wins[:, 4].sum(dtype=np.int64)),
              "kernel_ms": res["kernel_ms"],
              "model": "range: 32 B/range + 8 B/window block + 0.75 B/scored base",
              "ranges_call": {"api": "gac_score_ranges_device (windows searched on the device)",
                              "ms_per_step": res_r["step_ms"], "kernel_ms": res_r["kernel_ms"],
                              "same_bases": res_r["bases"] == res["bases"]},
              "roofline_step": roofline(algo, res["step_ms"], None,
                                        "whole call (plan + tile map + k_tile + fold)")}
    return kernel, roofline(algo, res["tile_ms"], pmc, "k_tile")


def scorechain_leg(legs, ch, steps, pmc):
    res = legs.run(None, True, steps)
    n, nb = ch["n"], ch["nb"]
    # SURVEY §8(d) full-chain model: 0.75 B/base + 12 B/block + 44 B/chain
    algo = 0.75 * res["bases"] + 12.0 * nb + 44.0 * n
    step = roofline(algo, res["step_ms"], None, "whole call (k_tile + cross-tile fold)")
    tile = roofline(algo, res["tile_ms"], pmc, "k_tile")
    return {"workload": "scoreChain: every C5 chain, global + local + aligned bases "
                        "(gac_score_chains_device)",
            "value": res["bases"] / (res["step_ms"] / 1e3) / 1e9, "unit": "Gbases/s",
            "ms_per_step": res["step_ms"], "steps": steps, "chains": n, "blocks": nb,
            "scored_bases": res["bases"], "kernel_ms": res["kernel_ms"],
            "model": "full chain: 0.75 B/base + 12 B/block + 44 B/chain",
            "roofline_step": step, "roofline": tile}


def scorechain_sharded_leg(d, ch, dist, rank, world, steps, expect=None):
    """N > 1: scoreChain's batch in the north-star form: chain-ID
    shards -- contiguous chain runs balanced by blocks, one per rank -- each
    scored whole on its rank's GPU (gac_score_chains_device into torch
    tensors), then ONE RCCL all-gather of {global, local, ali} over xGMI.  A
    step = scoring + all-gather, between barriers, max over ranks.  Rank 0
    checks the gathered set against the single-GPU scores (`expect`)."""
    import torch
    from genomealignmenttools_amd.gachain import GAC_Q, GAC_T, Engine, GapCosts
    from genomealignmenttools_amd.shard import (reduce_time_and_work, score_chains_sharded_gpu,
                                                shard_bounds)
    e = Engine(int(os.environ.get("LOCAL_RANK", "0")))
    e.load_2bit(GAC_T, os.path.join(d, "t.2bit"))
    e.load_2bit(GAC_Q, os.path.join(d, "q.2bit"))
    e.set_scoring(BLASTZ, GapCosts("loose"))
    names = lambda path: [ln.split()[0] for ln in open(path) if ln.strip()]
    tmap = np.array([e.seq_index(GAC_T, x) for x in names(os.path.join(d, "t.sizes"))], np.int32)
    qmap = np.array([e.seq_index(GAC_Q, x) for x in names(os.path.join(d, "q.sizes"))], np.int32)
    off = ch["off"]
    bounds = shard_bounds(np.diff(off), world)
    lo, hi = bounds[rank]
    b0, b1 = int(off[lo]), int(off[hi])
    cs = e.upload_chain_arrays(tmap[ch["tseq"][lo:hi]], qmap[ch["qseq"][lo:hi]],
                               ch["strand"][lo:hi], off[lo:hi + 1] - b0, ch["bt"][b0:b1],
                               ch["bq"][b0:b1], ch["bs"][b0:b1])
    n = ch["n"]
    for _ in range(3):
        res = score_chains_sharded_gpu(dist, rank, world, e, cs, n, bounds)
    torch.cuda.synchronize()
    dt = 0.0
    for _ in range(steps):
        dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        res = score_chains_sharded_gpu(dist, rank, world, e, cs, n, bounds)
        torch.cuda.synchronize()
        dt += time.perf_counter() - t0
    dt, _ = reduce_time_and_work(dist, dt, 0.0, device=f"cuda:{torch.cuda.current_device()}")
    step = dt / steps
    out = None
    if rank == 0:
        got = res.cpu().numpy()
        same = None
        if expect is not None:
            g, l, a = expect
            same = bool(np.array_equal(got[:, 0], g) and np.array_equal(got[:, 1], l)
                        and np.array_equal(got[:, 2], a))
        bases = int(ch["bs"].sum(dtype=np.int64))
        out = {"workload": "scoreChain: every C5 chain, global + local + aligned bases; chain-ID "
                           f"shards on {world} GPUs + one RCCL all-gather of (global, local, ali)",
               "value": bases / step / 1e9, "unit": "Gbases/s", "ms_per_step": step * 1e3,
               "steps": steps, "chains": n, "blocks": ch["nb"], "scored_bases": bases,
               "shard_chains": [hi_ - lo_ for lo_, hi_ in bounds],
               "allgather_bytes": 24 * max(hi_ - lo_ for lo_, hi_ in bounds) * world,
               "identical_to_single_gpu": same}
    cs.close()
    e.close()
    return out


PMC_PASSES = ("TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum",
              "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum")


def pmc_traffic(args, which):
    """HBM-side bytes per k_tile launch of one leg, measured in this run: two
    rocprofv3 --kernel-trace --pmc passes (no other trace domains; 3 and 2
    TCC counters) over a child process that makes the leg's call.  Bytes by
    request size, as MI355X_MICROARCH.md's HBM section prescribes for gfx950
    (not FETCH_SIZE): reads = 32 n32 + 64 n64 + 128 n128, writes = 64 n64 +
    32 (n - n64).  Run before this process touches the GPU.  Returns None on
    any failure (reported, never fatal)."""
    import csv
    import glob
    import shutil
    import tempfile
    if not shutil.which("rocprofv3"):
        return None
    child = [sys.executable, os.path.abspath(__file__), "--pmc-child", which, "--chains",
             str(args.chains), "--seed", str(args.seed), "--tmp", args.tmp]
    vals, durs = {}, []
    root = tempfile.mkdtemp(prefix="gac_pmc_", dir="/tmp")
    env = dict(os.environ, TMPDIR="/tmp")
    for i, counters in enumerate(PMC_PASSES):
        out = os.path.join(root, f"pass{i}")
        cmd = ["timeout", "-s", "KILL", "240", "rocprofv3", "--kernel-trace", "--pmc",
               *counters.split(), "--output-format", "csv", "-d", out, "-o", "run", "--", *child]
        r = subprocess.run(cmd, capture_output=True, text=True, cwd="/tmp", env=env, timeout=300)
        if r.returncode != 0:
            log(f"pmc {which} pass {i} rc={r.returncode}: {r.stderr[-800:]}")
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
            log(f"pmc {which} pass {i}: no k_tile rows")
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
    """The counter passes' workload: one leg's call, a few times."""
    d, _ = c5_files(args)
    ch = load_chains_bin(d)
    legs = Legs(d, ch)
    ranges = fills_windows(d) if args.pmc_child == "fills" else None
    legs.run(ranges, args.pmc_child == "scorechain", 3)
    legs.close()


# ---------------------------------------------------------------- CPU baseline
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


def _sample_chains(path, targets, dst):
    """The chains of `path` whose target is in `targets` (file order kept):
    their aligned bases up to the netting stop."""
    keep = set(targets)
    out, bases, stopped, cur = [], 0, False, None
    with open(path) as f:
        for line in f:
            if line.startswith("chain "):
                w = line.split()
                cur = w[2] in keep
                if cur:
                    out.append(line)
                    stopped = stopped or float(w[1]) < 0
            elif cur:
                out.append(line)
                if not stopped and line.strip():
                    bases += int(line.split()[0])
    with open(dst, "w") as f:
        f.writelines(out)
    return bases


def cpu_baseline_c5(d, ours):
    """The reference chainNet -rescore on a bounded sample of C5 (the chains on
    SAMPLE_TARGETS), one process; its target nets vs ours for those sequences."""
    p = lambda x: os.path.join(d, x)
    if not os.path.exists(REF_TOOL):
        return {"error": f"{REF_TOOL} not built (make ref)"}
    sample = p("sample.chain")
    bases = _sample_chains(p("in.chain"), SAMPLE_TARGETS, sample)
    ref = p("ref.sample")
    for o in (ref + ".t.net", ref + ".q.net"):
        if os.path.exists(o):
            os.remove(o)
    t0 = time.time()
    run_tool([REF_TOOL, sample, p("t.sizes"), p("q.sizes"), ref + ".t.net", ref + ".q.net",
              "-rescore", f"-tNibDir={p('t.2bit')}", f"-qNibDir={p('q.2bit')}", "-linearGap=loose"],
             [])
    t1 = time.time() - t0
    with open(ref + ".t.net") as f:
        rsec = _net_sections(f.read())[1]
    with open(ours + ".t.net") as f:
        osec = _net_sections(f.read())[1]
    same = all(rsec.get(k) == osec.get(k) and k in osec for k in SAMPLE_TARGETS)
    log(f"cpu baseline: reference chainNet -rescore on the {'+'.join(SAMPLE_TARGETS)} chains "
        f"{t1:.2f}s, target nets identical to ours: {same}")
    return {"value": bases / t1 / 1e9, "unit": "Gbases/s", "cores": 1, "kind": "reference",
            "seconds": t1, "identical_target_nets": same, "sample_aligned_bases": bases,
            "sample": f"reference chainNet -rescore (oracle/_ref, one process) on the C5 chains "
                      f"whose target is {' or '.join(SAMPLE_TARGETS)} (their netted aligned bases / "
                      f"wall time; their target-net sections compared with the headline's)"}


def _split_by_target(path, targets, dst):
    """One file per target in `targets` holding its chains (file order kept):
    {target: path}."""
    with open(path, "rb") as f:
        data = f.read()
    pieces = data.split(b"\nchain ")  # each piece: a chain without "chain " and its last newline
    del data
    if pieces[0].startswith(b"chain "):
        pieces[0] = pieces[0][6:]
    else:  # '#' lines before the first chain
        pieces = pieces[1:]
    last = len(pieces) - 1
    keep = {t.encode(): [] for t in targets}
    for k, p in enumerate(pieces):
        i = p.find(b" ")
        sel = keep.get(p[i + 1:p.find(b" ", i + 1)])
        if sel is not None:
            sel.append(b"chain " + p + (b"\n" if k < last else b""))
    out = {}
    for t, chunks in keep.items():
        name = os.path.join(dst, f"allcores.{t.decode()}.chain")
        with open(name, "wb") as f:
            f.writelines(chunks)
        out[t.decode()] = name
    return out


def _target_bases(d, targets):
    """Aligned bases, up to the netting stop (the headline's measure), of the
    chains whose target is in `targets`, from chains.bin."""
    ch = load_chains_bin(d)
    with open(os.path.join(d, "t.sizes")) as f:
        names = [line.split()[0] for line in f if line.strip()]
    ids = np.array([names.index(t) for t in targets if t in names], np.int32)
    neg = np.flatnonzero(ch["score"] < 0)
    stop = int(neg[0]) if len(neg) else ch["n"]
    cs = np.concatenate([[0], np.cumsum(ch["bs"], dtype=np.int64)])
    per = cs[ch["off"][1:stop + 1]] - cs[ch["off"][:stop]]
    return int(per[np.isin(ch["tseq"][:stop], ids)].sum())


def cpu_baseline_all_cores(d, cores):
    """The reference chainNet -rescore on ALL_CORES_TARGETS' chains, one process
    per target sequence, `cores` of them at a time: the chains' aligned bases up
    to the netting stop / wall time."""
    p = lambda x: os.path.join(d, x)
    files = _split_by_target(p("in.chain"), ALL_CORES_TARGETS, d)
    jobs = sorted(files.items(), key=lambda kv: -os.path.getsize(kv[1]))  # largest first
    t0 = time.time()
    running, done = [], []
    while jobs or running:
        while jobs and len(running) < cores:
            t, f = jobs.pop(0)
            o = p(f"allcores.{t}")
            pr = subprocess.Popen([REF_TOOL, f, p("t.sizes"), p("q.sizes"), o + ".t.net",
                                   o + ".q.net", "-rescore", f"-tNibDir={p('t.2bit')}",
                                   f"-qNibDir={p('q.2bit')}", "-linearGap=loose"],
                                  stdout=subprocess.DEVNULL, stderr=subprocess.PIPE)
            running.append((t, o, pr))
        time.sleep(0.05)
        for item in list(running):
            if item[2].poll() is not None:
                running.remove(item)
                if item[2].returncode != 0:
                    raise RuntimeError(f"reference chainNet on {item[0]}: "
                                       f"{item[2].stderr.read()[-300:]!r}")
                done.append(item)
    wall = time.time() - t0
    bases = _target_bases(d, [t for t, _, _ in done])
    for _, o, _ in done:
        for x in (o + ".t.net", o + ".q.net"):
            os.remove(x)
    for f in files.values():
        os.remove(f)
    return {"value": bases / wall / 1e9, "unit": "Gbases/s", "cores": cores, "kind": "reference",
            "seconds": wall, "sample_aligned_bases": bases,
            "sample": f"reference chainNet -rescore (oracle/_ref) on the C5 chains of "
                      f"{len(done)} target sequences ({ALL_CORES_TARGETS[0]}..{ALL_CORES_TARGETS[-1]}), "
                      f"one process per sequence, {cores} at a time; value = their chains' aligned bases "
                      f"up to the netting stop (the headline's measure) / wall time"}


def scorechain_e2e_leg(d, info, steps, ref_sample):
    """bin/scoreChain end to end on C5 (every chain rescored: global score,
    written as chain text), input aligned bases / wall time; with
    ref_sample, the reference scoreChain on the cpu baseline's sample chains
    (one process) against ours on the same file."""
    p = lambda x: os.path.join(d, x)
    out = p("ours.sc.chain")
    cmd = [SC_TOOL, p("in.chain"), p("t.2bit"), p("q.2bit"), out, "-linearGap=loose"]
    run_tool(cmd, [out])  # warmup
    dt = 0.0
    for _ in range(steps):
        if os.path.exists(out):
            os.remove(out)
        t0 = time.perf_counter()
        run_tool(cmd, [])
        dt += time.perf_counter() - t0
    dt /= steps
    parity = full_parity("c5", {"in_chain_sha256": p("in.chain"), "scorechain.chain_sha256": out})
    os.remove(out)
    r = run_tool(cmd + ["-verbose=2"], [], env=dict(os.environ, GAC_TIMING="1"))
    res = {"workload": "scoreChain end to end (bin/scoreChain), C5 whole genome: every chain's "
                       "score rescored and the chain file rewritten",
           "value": info["input_aligned_bases"] / dt / 1e9, "unit": "Gbases/s",
           "ms_per_step": dt * 1e3, "steps": steps, "parity_full": parity,
           "tool_stages": [x.strip() for x in r.stderr.splitlines()
                           if x.startswith(("[stage]", "[gac_chains_upload]", "[gt_read_chains]"))]}
    os.remove(out)
    if ref_sample and os.path.exists(REF_SC_TOOL) and os.path.exists(p("sample.chain")):
        sample, ro, oo = p("sample.chain"), p("ref.sample.sc.chain"), p("ours.sample.sc.chain")
        t0 = time.time()
        run_tool([REF_SC_TOOL, sample, p("t.2bit"), p("q.2bit"), ro, "-linearGap=loose"], [ro])
        t1 = time.time() - t0
        run_tool([SC_TOOL, sample, p("t.2bit"), p("q.2bit"), oo, "-linearGap=loose"], [oo])
        bases = 0
        with open(sample) as f:
            for line in f:
                w = line.split()
                if len(w) in (1, 3) and w[0].isdigit():
                    bases += int(w[0])
        res["cpu_reference"] = {"seconds": t1, "cores": 1, "kind": "reference",
                                "value": bases / t1 / 1e9, "sample_aligned_bases": bases,
                                "identical_output": filecmp.cmp(ro, oo, False),
                                "sample": "reference scoreChain (oracle/_ref) on the cpu "
                                          "baseline's sample chains"}
        log(f"scoreChain: ours {dt * 1e3:.0f} ms on C5; reference {t1:.2f}s on the sample "
            f"({bases / 1e6:.0f} M bases), identical: {res['cpu_reference']['identical_output']}")
    return res


# ---------------------------------------------------------------- full-scale parity
GOLDEN_FULL = os.path.join(REPO, "tests", "golden", "fullscale")


def sha256_files(paths):
    """sha256 of several files at once (one thread each; hashlib drops the
    GIL on large buffers): {path: hexdigest}."""
    import hashlib
    from concurrent.futures import ThreadPoolExecutor

    def one(path):
        h = hashlib.sha256()
        with open(path, "rb") as f:
            for b in iter(lambda: f.read(1 << 24), b""):
                h.update(b)
        return h.hexdigest()
    with ThreadPoolExecutor(len(paths)) as ex:
        return dict(zip(paths, ex.map(one, paths)))


def full_parity(which, files):
    """The outputs of a full-size run against the reference's sha256
    (tests/golden/fullscale/<which>.json, made by the reference on the same
    seeded input by tests/golden/make_fullscale_golden.py).  files: {golden
    key ("a.b" = nested): path}.  Returns {"identical": all equal, per key
    {"ours", "reference", "same"}} -- checked outside every timed region."""
    with open(os.path.join(GOLDEN_FULL, f"{which}.json")) as f:
        gold = json.load(f)
    t0 = time.time()
    got = sha256_files(list(files.values()))
    res, same = {}, True
    for key, path in files.items():
        ref = gold
        for k in key.split("."):
            ref = ref[k]
        ok = got[path] == ref
        same = same and ok
        res[key] = {"ours": got[path], "reference": ref, "same": ok}
    res["identical"] = same
    ins = [k for k in files if k.startswith("in_")]
    if ins and not all(res[k]["same"] for k in ins):
        # another seed or size than the golden's: nothing to compare against
        res["identical"] = None
        res["unpinned"] = "input differs from the golden's (another --seed / size): parity unpinned"
    res["golden"] = f"tests/golden/fullscale/{which}.json ({gold['generator']}; reference run on "
    res["golden"] += f"{gold['reference_host']})"
    res["hash_seconds"] = round(time.time() - t0, 2)
    return res


def c4_files(args):
    """C4: gac_synth c4, 50 M PSL blocks over 24 x 21 pairs x 2
    strands, seed 7; written once per box under --tmp (~20 s)."""
    d = os.path.join(args.tmp, f"gac_bench_c4_{args.c4_blocks}_7")
    if not os.path.exists(os.path.join(d, "info.json")):
        t0 = time.time()
        subprocess.run([SYNTH, "c4", d, "-seed=7", f"-blocks={args.c4_blocks}",
                        f"-threads={min(host_threads(), 32)}"], check=True)
        log(f"C4: written in {time.time() - t0:.1f}s")
    with open(os.path.join(d, "info.json")) as f:
        return d, json.load(f)


def c4_leg(args, dist, world, rank, local, barrier, step_env):
    """configs[3]: axtChain -psl on C4 (50 M PSL blocks), 1 GPU, and at N > 1
    chain-sharded: every rank runs axtChain -nranks=N -rank=r -gpu=LOCAL_RANK
    (seqPairs dealt by block count, rank 0 merges and writes).  One warmup +
    `steps` timed runs between barriers, max over ranks; the output's sha256
    against the reference's (tests/golden/fullscale/c4.json)."""
    d, info = c4_files(args) if rank == 0 else (None, None)
    barrier()
    if rank != 0:
        d, info = c4_files(args)
    p = lambda x: os.path.join(d, x)
    out = p(f"ours.r{world}.chain")
    cmd = [AXT_TOOL, "-linearGap=loose", "-verbose=0", "-psl", p("in.psl"), p("t.2bit"), p("q.2bit"),
           out]
    if world > 1:
        cmd += [f"-nranks={world}", f"-rank={rank}", f"-gpu={local}"]
    dt = 0.0
    for k in range(1 + args.c4_steps):
        if rank == 0 and os.path.exists(out):
            os.remove(out)
        barrier()
        t0 = time.perf_counter()
        run_tool(cmd, [], env=step_env())
        barrier()
        if k:
            dt += time.perf_counter() - t0
    if dist is not None:
        from genomealignmenttools_amd.shard import reduce_time_and_work
        dt, _ = reduce_time_and_work(dist, dt, 0.0, device="cpu" if os.environ.get(
            "GAC_BENCH_ONE_GPU") else f"cuda:{local}")
    if rank != 0:
        return None
    dt /= max(args.c4_steps, 1)
    with open(os.path.join(GOLDEN_FULL, "c4.json")) as f:
        gold = json.load(f)
    res = {"workload": "configs[3]: axtChain -psl end to end (bin/axtChain) on C4, "
                       + ("1 GPU" if world == 1 else f"{world} GPUs, seqPairs sharded (-nranks)"),
           "blocks": info["blocks"], "pairs": info["pairs"],
           "largest_pair_blocks": info["largest_pair_blocks"], "value": info["blocks"] / dt / 1e6,
           "unit": "M PSL blocks chained/s", "ms_per_step": dt * 1e3, "steps": args.c4_steps,
           "reference": {"seconds": gold["axtchain"]["reference_seconds"],
                         "host": gold["reference_host"], "kind": "reference (oracle/_ref/axtChain)"}}
    if args.c4_blocks == gold["info"]["blocks"] or args.c4_blocks == 50_000_000:
        res["parity_full"] = full_parity("c4", {"in_psl_sha256": p("in.psl"),
                                                "axtchain.chain_sha256": out})
    os.remove(out)
    if world == 1 and not args.no_c4_ref:
        try:
            res["reference_on_box"] = c4_ref_sample(d)
        except Exception as ex:  # (reported, never fatal)
            res["reference_on_box"] = {"error": str(ex)[:300]}
    return res


def c4_ref_sample(d):
    """The reference axtChain (oracle/_ref, one process, test
    infrastructure) timed on this host on a pair subset of C4: the PSL
    records whose target is chr4 (42 of the 1008 seqPairs, ~0.33 M of the
    50 M blocks), with ours on the same file and the two outputs compared.
    The reference's whole-C4 time (1287 s, build container) is dominated by
    the 11.5 M-block pair, whose DP cost grows faster than linearly, so this
    sample's per-block rate overstates the reference's whole-set rate."""
    if not os.path.exists(REF_AXT_TOOL):
        return {"error": f"{REF_AXT_TOOL} not built (make ref)"}
    p = lambda x: os.path.join(d, x)
    sample = p("sample_chr4.psl")
    if not os.path.exists(sample):
        with open(sample + ".tmp", "w") as f:
            subprocess.run(["awk", "-F\t", '$14=="chr4"', p("in.psl")], stdout=f, check=True,
                           timeout=600)
        os.replace(sample + ".tmp", sample)
    blocks = 0
    with open(sample) as f:
        for line in f:
            blocks += int(line.split("\t", 18)[17])
    args_ = ["-linearGap=loose", "-verbose=0", "-psl", sample, p("t.2bit"), p("q.2bit")]
    t0 = time.perf_counter()
    run_tool([REF_AXT_TOOL] + args_ + [p("sample.ref.chain")], [])
    t_ref = time.perf_counter() - t0
    run_tool([AXT_TOOL] + args_ + [p("sample.ours.chain")], [])  # (warm)
    t0 = time.perf_counter()
    run_tool([AXT_TOOL] + args_ + [p("sample.ours.chain")], [])
    t_ours = time.perf_counter() - t0
    same = filecmp.cmp(p("sample.ref.chain"), p("sample.ours.chain"), shallow=False)
    for x in ("sample.ref.chain", "sample.ours.chain"):
        os.remove(p(x))
    return {"sample": "C4 PSL records with target chr4 (every query, both strands)",
            "blocks": blocks, "reference_seconds": t_ref, "ours_seconds": t_ours,
            "reference_Mblocks_per_s": blocks / t_ref / 1e6, "identical": same,
            "cores": 1, "kind": "reference (oracle/_ref/axtChain), this host",
            "cpu_model": host_cpu()["cpu_model"]}


def c2_leg(args, steps, warmup):
    d, info = c2_files(args)
    out = os.path.join(d, "ours")
    outs = [out + ".t.net", out + ".q.net"]
    cmd = tool_cmd(d, out, 1, 0)
    for _ in range(warmup):
        run_tool(cmd, outs)
    dt = 0.0
    for _ in range(steps):  # (outputs removed outside the clock, as in the headline)
        for o in outs:
            if os.path.exists(o):
                os.remove(o)
        t0 = time.perf_counter()
        run_tool(cmd, [])
        dt += time.perf_counter() - t0
    dt /= steps
    res = {"workload": "configs[1]: chainNet -rescore end to end on C2 (hg38 chr1 x mm10)",
           "value": info["netted_aligned_bases"] / dt / 1e9, "unit": "Gbases/s",
           "ms_per_step": dt * 1e3, "steps": steps, **info,
           "tool_stages": staged_run(d, out)}  # (one more, untimed, with the stage laps)
    if not args.no_cpu_baseline and os.path.exists(REF_TOOL):
        p = lambda x: os.path.join(d, x)
        ref = p("ref")
        for o in (ref + ".t.net", ref + ".q.net"):
            if os.path.exists(o):
                os.remove(o)
        t0 = time.time()
        run_tool([REF_TOOL, p("in.chain"), p("t.sizes"), p("q.sizes"), ref + ".t.net",
                  ref + ".q.net", "-rescore", f"-tNibDir={p('t.2bit')}", f"-qNibDir={p('q.2bit')}",
                  "-linearGap=loose"], [])
        t1 = time.time() - t0
        same = (filecmp.cmp(out + ".t.net", ref + ".t.net", False)
                and filecmp.cmp(out + ".q.net", ref + ".q.net", False))
        res["cpu_reference"] = {"seconds": t1, "cores": 1, "identical_nets": same,
                                "value": info["netted_aligned_bases"] / t1 / 1e9}
        log(f"C2: ours {dt * 1e3:.1f} ms, reference {t1:.2f}s, nets identical: {same}")
    return res


CC_TOOL = os.path.join(PKG, "bin", "chainCleaner")
REF_CC_TOOL = os.path.join(REPO, "oracle", "_ref", "chainCleaner")


def c3_files(args):
    """C3 (configs[2]): the C2 shape (hg38 chr1 x mm10, 200 k chains) plus
    1000 planted chain-breaking loci (synth.c3_case, as
    tests/test_gpu_configs.py::test_c3_chaincleaner), header scores from
    bin/scoreChain, sorted and numbered, and the reference pipeline's net
    (chainNet -minScore=0 | NetFilterNonNested.perl -minScore1 3000; the
    reference chainNet when it is built, else ours -- byte-identical).
    Written once per box under --tmp."""
    d = os.path.join(args.tmp, "gac_bench_c3_42")
    p = lambda x: os.path.join(d, x)
    if os.path.exists(p("info.json")):
        with open(p("info.json")) as f:
            return d, json.load(f)
    from genomealignmenttools_amd import chainfile, synth
    os.makedirs(d, exist_ok=True)
    t0 = time.time()
    tg, qg, ca = synth.c3_case(seed=42, n_chains=200_000, n_loci=1000)
    synth.write_2bit(tg, p("t.2bit"))
    synth.write_2bit(qg, p("q.2bit"))
    synth.write_sizes(tg.sizes, p("t.sizes"))
    synth.write_sizes(qg.sizes, p("q.sizes"))
    chainfile.write_chains_fast(ca, p("unscored.chain"))
    del tg, qg, ca
    run_tool([SC_TOOL, p("unscored.chain"), p("t.2bit"), p("q.2bit"), p("sc.chain"),
              "-linearGap=loose"], [])
    sc = chainfile.read_chains(p("sc.chain"))
    sc = sc.subset(np.argsort(-sc.score, kind="stable"))
    sc.id = np.arange(1, sc.n + 1, dtype=np.int64)
    chainfile.write_chains_fast(sc, p("in.chain"))
    info = {"chains": int(sc.n), "blocks": int(sc.blk_off[-1]), "planted_loci": 1000}
    del sc
    net_tool = REF_TOOL if os.path.exists(REF_TOOL) else os.path.join(PKG, "bin", "chainNet")
    net = subprocess.run([net_tool, "-minScore=0", p("in.chain"), p("t.sizes"), p("q.sizes"),
                          "stdout", "/dev/null"], capture_output=True, check=True)
    filt = subprocess.run([os.path.join(PKG, "bin", "NetFilterNonNested.perl"), "/dev/stdin",
                           "-minScore1", "3000"], input=net.stdout, capture_output=True, check=True)
    with open(p("in.net"), "wb") as f:
        f.write(filt.stdout)
    info["net_from"] = "reference chainNet" if net_tool == REF_TOOL else "bin/chainNet"
    for x in ("unscored.chain", "sc.chain"):
        os.remove(p(x))
    with open(p("info.json"), "w") as f:
        json.dump(info, f)
    log(f"C3: written in {time.time() - t0:.1f}s")
    return d, info


def c3_leg(args, steps):
    """configs[2]: bin/chainCleaner -net= end to end on C3 (the suspect-block
    rescoring on the GPU, the replay of the reference's decisions on the
    host), `steps` timed runs (outputs removed outside the clock), then the
    reference chainCleaner on the same files, timed, and the outputs
    (chains, removedSuspects.bed) compared byte for byte outside every
    clock."""
    d, info = c3_files(args)
    p = lambda x: os.path.join(d, x)
    opts = [f"-net={p('in.net')}", "-linearGap=loose"]
    outs = [p("ours.chain"), p("ours.bed")]
    cmd = [CC_TOOL, p("in.chain"), p("t.2bit"), p("q.2bit")] + outs + opts
    run_tool(cmd, outs)  # warmup
    dt = 0.0
    for _ in range(steps):
        for o in outs:
            if os.path.exists(o):
                os.remove(o)
        t0 = time.perf_counter()
        run_tool(cmd, [])
        dt += time.perf_counter() - t0
    dt /= steps
    r = run_tool(cmd + ["-verbose=2"], [], env=dict(os.environ, GAC_TIMING="1"))
    with open(p("ours.bed")) as f:
        removed = sum(1 for _ in f)
    res = {"workload": "configs[2]: chainCleaner -net= end to end (bin/chainCleaner) on C3: the "
                       "C2 chain set + 1000 planted chain-breaking loci",
           "ms_per_step": dt * 1e3, "steps": steps, **info, "removed_suspects": removed,
           "tool_stages": [x.strip() for x in r.stderr.splitlines()
                           if x.startswith(("[stage]", "GPU:", "[gac_chains_upload]"))]}
    if os.path.exists(REF_CC_TOOL):
        ro = [p("ref.chain"), p("ref.bed")]
        for o in ro:
            if os.path.exists(o):
                os.remove(o)
        env = dict(os.environ, PATH=os.path.dirname(REF_CC_TOOL) + os.pathsep + os.environ["PATH"])
        t0 = time.time()
        run_tool([REF_CC_TOOL, p("in.chain"), p("t.2bit"), p("q.2bit")] + ro + opts, [], env=env)
        t1 = time.time() - t0
        same = filecmp.cmp(outs[0], ro[0], False) and filecmp.cmp(outs[1], ro[1], False)
        res["reference"] = {"seconds": t1, "cores": 1, "kind": "reference (oracle/_ref/chainCleaner)"}
        res["identical"] = same
        res["speedup_vs_reference"] = t1 / dt
        log(f"C3: ours {dt * 1e3:.0f} ms, reference {t1:.2f}s, outputs identical: {same}")
    else:
        res["identical"] = None
    return res


# ---------------------------------------------------------------- main
def main():
    args = parse()
    if args.gen_only:
        c5_files(args)
        return
    if args.pmc_child:
        pmc_child(args)
        return
    maybe_self_launch(args)
    if args.launch_check:
        dist, world, rank, local, one_gpu, group = init_ranks(args)
        if rank == 0:
            print(json.dumps({"launch_check": True, "n_gpus": world,
                              "process_group": group}), flush=True)
        if dist is not None:
            dist.barrier()
            dist.destroy_process_group()
        return
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    d = info = None
    if rank == 0:  # generated before any process opens a device
        d, info = c5_files(args)
    dist, world, rank, local, one_gpu, group = init_ranks(args)
    rdist = None
    if world == 1 and args.sharded_scorechain:
        # rehearsal of the N > 1 scoreChain leg: a world-1 RCCL group, made
        # before this process opens the device through libgachain (torch's
        # HIP initialisation fails after it)
        import socket
        import torch
        import torch.distributed as rdist
        s_ = socket.socket()
        s_.bind(("127.0.0.1", 0))
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(s_.getsockname()[1]))
        s_.close()
        torch.cuda.set_device(0)
        rdist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda:0"))

    def barrier():
        if dist is not None:
            dist.barrier()

    barrier()
    if rank != 0:
        d, info = c5_files(args)  # written by rank 0 (same node)
    out_base = os.path.join(d, f"ours.r{world}")
    outs = [out_base + ".t.net", out_base + ".q.net"]
    ch = None
    stages = pmc_f = pmc_s = None
    if rank == 0 and world == 1:
        stages = staged_run(d, out_base)  # also dumps the fills for the kernel leg
        if not (args.no_pmc or args.no_kernel):
            pmc_f = pmc_traffic(args, "fills")
            if not args.no_scorechain:
                pmc_s = pmc_traffic(args, "scorechain")

    cmd = tool_cmd(d, out_base, world, rank)
    # every rank of one step shares a marker token (tells this step's part
    # markers from an earlier, failed one's; see gt_ranks_place)
    run_id = f"{os.environ.get('TORCHELASTIC_RUN_ID', 'x')}-{os.environ.get('MASTER_PORT', '0')}"
    step_no = [0]

    # host threads per rank (rank_tool_threads: the launcher's setting, not
    # torch.distributed.run's OMP_NUM_THREADS=1 default, else this process's
    # usable cores shared by the node's ranks)
    tool_threads = rank_tool_threads(world, os.environ, usable_cpus())

    def step_env():
        step_no[0] += 1
        return dict(os.environ, GAC_RANK_TOKEN=f"{run_id}-{step_no[0]}", **tool_threads)

    for _ in range(args.warmup):
        barrier()
        run_tool(cmd, outs if rank == 0 else [], env=step_env())
    # Each step is timed between barriers; the previous step's output files
    # are removed before the step's clock starts (unlinking ~1.5 GB of nets
    # frees their page cache: 0.3-0.6 s that is the harness's, not the
    # tool's -- the reference baseline is timed the same way).
    dt = 0.0
    step_ms = []
    for _ in range(args.steps):
        if rank == 0:
            for o in outs:
                if os.path.exists(o):
                    os.remove(o)
        barrier()
        t0 = time.perf_counter()
        run_tool(cmd, [], env=step_env())
        barrier()  # rank 0 finishes last (it waits for every part)
        dt += time.perf_counter() - t0
        step_ms.append(round(1e3 * (time.perf_counter() - t0), 1))
    if dist is not None:
        from genomealignmenttools_amd.shard import reduce_time_and_work
        dev = "cpu" if one_gpu else f"cuda:{local}"
        dt, _ = reduce_time_and_work(dist, dt, 0.0, device=dev)
    step_s = dt / args.steps
    parity = None
    if rank == 0:  # (outside the timed region)
        parity = full_parity("c5", {"in_chain_sha256": os.path.join(d, "in.chain"),
                                    "chainnet_rescore.t_net_sha256": outs[0],
                                    "chainnet_rescore.q_net_sha256": outs[1]})
        log(f"C5 nets identical to the reference's (sha256): {parity['identical']}")
    out = {
        "metric": METRIC,
        "value": info["netted_aligned_bases"] / step_s / 1e9,
        "unit": "Gbases/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": step_s * 1e3, "step_ms_rank0": step_ms, "higher_is_better": True,
        "scaling": "strong", "vs_baseline": None, "dtype": "int64",
        "data": "synthetic (seeded C5 by gac_synth: all 455 hg38 x 66 mm10 sequences at their "
                "real sizes, planted chains; no real genomes)",
        "config": {"workload": "chainNet -rescore end to end (bin/chainNet), C5 whole genome"
                               + ("" if world == 1 else f", chromosome sides split over {world} ranks"),
                   **info, "parallelism": f"chromosome-side shards x{world}",
                   "host_threads_per_rank": int(tool_threads.get("GAC_THREADS", host_threads())),
                   "tool_stages": stages},
        # the group as torch.distributed (RCCL) saw it: n_gpus above is its size
        "process_group": group or {"backend": None, "world_size": 1,
                                   "ranks": [{"rank": 0, "local_rank": 0, "device": "cuda:0"}]},
        # both nets of the last timed step vs the reference's on the whole C5
        "parity_full": parity,
        "identical_nets_full": parity["identical"] if parity else None,
    }
    if one_gpu:
        out["rehearsal"] = "GAC_BENCH_ONE_GPU: every rank on device 0 over gloo (not a GPU curve)"
    if rank == 0 and world == 1 and not args.no_c2:
        try:
            out["c2"] = c2_leg(args, args.c2_steps, 1)
        except Exception as ex:  # reported, never fatal
            out["c2"] = {"error": str(ex)[:300]}
    if rank == 0 and world == 1 and not args.no_c3:
        try:
            out["c3"] = c3_leg(args, args.c3_steps)
        except Exception as ex:  # (reported, never fatal to the headline)
            out["c3"] = {"error": str(ex)[:300]}
    if not args.no_c4:
        try:
            c4 = c4_leg(args, dist, world, rank, local, barrier, step_env)
        except Exception as ex:  # reported, never fatal
            c4 = {"error": str(ex)[:300]}
        if rank == 0:
            out["c4"] = c4
    expect = None
    if rank == 0 and not args.no_kernel:
        if world > 1 and not os.path.exists(os.path.join(d, "fills.bin")):
            staged_run(d, os.path.join(d, "ours.fills"))  # untimed, after the timed region
        ch = load_chains_bin(d)
        legs = Legs(d, ch)
        out["kernel"], out["roofline"] = fills_leg(legs, d, ch, args.kernel_steps, pmc_f)
        if not args.no_scorechain:
            if world == 1:
                out["scorechain"] = scorechain_leg(legs, ch, args.kernel_steps, pmc_s)
            else:
                expect = legs.score_all()
        legs.close()
    if world > 1 and not (args.no_kernel or args.no_scorechain or one_gpu):
        barrier()
        if ch is None:
            ch = load_chains_bin(d)
        sc = scorechain_sharded_leg(d, ch, dist, rank, world, args.kernel_steps, expect)
        if rank == 0:
            out["scorechain"] = sc
    elif rdist is not None:  # rehearsal of the N > 1 leg on one GPU
        legs = Legs(d, ch if ch is not None else load_chains_bin(d))
        expect = legs.score_all()
        legs.close()
        out["scorechain_sharded"] = scorechain_sharded_leg(d, ch if ch is not None else
                                                           load_chains_bin(d), rdist, 0, 1,
                                                           args.kernel_steps, expect)
        rdist.destroy_process_group()
    if rank == 0 and world == 1 and not args.no_kernel:
        ceil = gather_ceiling()
        out["gather_ceiling"] = ceil
        add_ceiling(out.get("roofline"), ceil)
        add_ceiling((out.get("scorechain") or {}).get("roofline"), ceil)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            out["cpu_baseline"] = cpu_baseline_c5(d, out_base)
        except Exception as ex:  # reported, never fatal
            out["cpu_baseline"] = {"error": str(ex)[:300]}
        out["cpu_baseline"].update(host_cpu())
        try:  # how the sample's rate relates to the whole genome's (same host, golden run)
            with open(os.path.join(GOLDEN_FULL, "c5.json")) as f:
                g = json.load(f)
            whole = g["info"]["netted_aligned_bases"] / g["chainnet_rescore"]["reference_seconds"]
            samp = g["reference_sample_chr21_chr22"]
            srate = samp["netted_aligned_bases"] / samp["seconds"]
            out["cpu_baseline"]["whole_c5_reference"] = {
                "seconds": g["chainnet_rescore"]["reference_seconds"], "host": g["reference_host"],
                "value": whole / 1e9, "sample_value_same_host": srate / 1e9,
                "whole_over_sample_rate": whole / srate,
                "note": "the reference chainNet -rescore on the whole C5 input (its nets are the "
                        "full-scale parity golden); the sample rate above overstates the "
                        "reference's whole-genome rate by 1/whole_over_sample_rate"}
        except (OSError, KeyError, ValueError) as ex:
            out["cpu_baseline"]["whole_c5_reference"] = {"error": str(ex)[:200]}
        try:
            out["cpu_baseline"]["all_cores"] = cpu_baseline_all_cores(
                d, min(16, host_threads(), len(ALL_CORES_TARGETS)))
        except Exception as ex:  # reported, never fatal
            out["cpu_baseline"]["all_cores"] = {"error": str(ex)[:300]}
    if rank == 0 and world == 1 and not args.no_scorechain:
        try:
            out["scorechain_e2e"] = scorechain_e2e_leg(d, info, 2, not args.no_cpu_baseline)
        except Exception as ex:  # reported, never fatal
            out["scorechain_e2e"] = {"error": str(ex)[:300]}
    if rank == 0:
        print(json.dumps(out), flush=True)
    barrier()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
