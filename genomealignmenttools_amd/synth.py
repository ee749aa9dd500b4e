"""Seeded synthetic genomes and chain sets.

Genomes are produced directly in the .2bit code (T=0 C=1 A=2 G=3), with N
runs and soft-mask runs, and can be written as real .2bit files.  Chains are
planted homology: query bases under each block are a mutated copy of the
target (12% substitutions, transitions:transversions 2:1), '-' strand chains
write the reverse complement.  Everything is numpy-vectorised so the C2 set
(~2e5 chains, ~2e8 aligned bases, hg38 chr1 x mm10) builds in seconds.
"""
from __future__ import annotations

import os
import struct
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

import numpy as np

from .chainfile import ChainArrays

_NT = np.frombuffer(b"tcag", dtype=np.uint8)

# loose gap table (kent/src/lib/gapCalc.c:51-57) -- only used for the
# approximate synthetic header score, never for scoring
_LOOSE_POS = np.array([1, 2, 3, 11, 111, 2111, 12111, 32111, 72111, 152111, 252111], float)
_LOOSE_Q = np.array([325, 360, 400, 450, 600, 1100, 3600, 7600, 15600, 31600, 56600], float)
_LOOSE_B = np.array([625, 660, 700, 750, 900, 1400, 4000, 8000, 16000, 32000, 57000], float)

# blastz default, [query][target] in 2bit code order (T, C, A, G)
_BLASTZ_ACGT = np.array([[91, -114, -31, -123], [-114, 100, -125, -31],
                         [-31, -125, 100, -114], [-123, -31, -114, 91]], np.int64)
_CODE2ACGT = np.array([3, 1, 0, 2])


def matrix_by_code(mat_acgt: np.ndarray) -> np.ndarray:
    m = np.asarray(mat_acgt, np.int64)
    return m[np.ix_(_CODE2ACGT, _CODE2ACGT)]


@dataclass
class Genome:
    names: List[str]
    codes: List[np.ndarray]                      # uint8 per base, 0..3
    nruns: List[Tuple[np.ndarray, np.ndarray]]   # (starts, sizes) int32
    mruns: List[Tuple[np.ndarray, np.ndarray]] = field(default_factory=list)

    @property
    def sizes(self) -> Dict[str, int]:
        return {n: len(c) for n, c in zip(self.names, self.codes)}

    def index(self, name: str) -> int:
        return self.names.index(name)

    def packed(self, i: int) -> np.ndarray:
        """.2bit payload bytes (2 bits/base, MSB first)."""
        c = self.codes[i]
        n = len(c)
        pad = (-n) % 4
        if pad:
            c = np.concatenate([c, np.zeros(pad, np.uint8)])
        c = c.reshape(-1, 4)
        return ((c[:, 0] << 6) | (c[:, 1] << 4) | (c[:, 2] << 2) | c[:, 3]).astype(np.uint8)

    def text(self, i: int) -> str:
        """Decoded 'acgtn' text (reference twoBitReadSeqFrag without mask case)."""
        s = _NT[self.codes[i]].copy()
        st, sz = self.nruns[i]
        for a, b in zip(st, sz):
            s[a:a + b] = ord("n")
        return s.tobytes().decode()

    def seq_records(self):
        """(name, size, packed, n_starts, n_sizes) for Engine.add_sequences."""
        for i, n in enumerate(self.names):
            yield n, len(self.codes[i]), self.packed(i), self.nruns[i][0], self.nruns[i][1]


def random_runs(rng, size: int, frac: float, mean_len: int) -> Tuple[np.ndarray, np.ndarray]:
    if frac <= 0 or size < 4:
        return np.zeros(0, np.int32), np.zeros(0, np.int32)
    k = max(1, int(size * frac / mean_len))
    starts = np.sort(rng.integers(0, size, k))
    lens = rng.geometric(1.0 / mean_len, k)
    ends = np.minimum(starts + lens, size)
    # merge overlaps -> disjoint sorted runs
    out_s, out_e = [], []
    cs, ce = int(starts[0]), int(ends[0])
    for s, e in zip(starts[1:], ends[1:]):
        if s <= ce:
            ce = max(ce, int(e))
        else:
            out_s.append(cs)
            out_e.append(ce)
            cs, ce = int(s), int(e)
    out_s.append(cs)
    out_e.append(ce)
    s = np.asarray(out_s, np.int32)
    return s, (np.asarray(out_e, np.int32) - s)


def random_genome(sizes: Dict[str, int], seed: int, n_frac: float = 0.005,
                  n_mean: int = 2000, mask_frac: float = 0.0) -> Genome:
    rng = np.random.default_rng(seed)
    names, codes, nr, mr = [], [], [], []
    for name, size in sizes.items():
        names.append(name)
        b = np.frombuffer(rng.bytes((size + 3) // 4), dtype=np.uint8)
        c = np.empty(b.size * 4, np.uint8)
        c[0::4] = b >> 6
        c[1::4] = (b >> 4) & 3
        c[2::4] = (b >> 2) & 3
        c[3::4] = b & 3
        c = c[:size].copy()
        ns, nz = random_runs(rng, size, n_frac, n_mean)
        for a, l in zip(ns, nz):
            c[a:a + l] = 0  # .2bit stores N as T
        codes.append(c)
        nr.append((ns, nz))
        mr.append(random_runs(rng, size, mask_frac, 300) if mask_frac > 0 else
                  (np.zeros(0, np.int32), np.zeros(0, np.int32)))
    return Genome(names, codes, nr, mr)


def write_2bit(g: Genome, path: str) -> None:
    """Write a version-0 .2bit file (kent twoBit.c layout)."""
    n = len(g.names)
    header = struct.pack("<IIII", 0x1A412743, 0, n, 0)
    index_size = sum(1 + len(nm.encode()) + 4 for nm in g.names)
    off = len(header) + index_size
    recs, index = [], []
    for i, nm in enumerate(g.names):
        size = len(g.codes[i])
        ns, nz = g.nruns[i]
        ms, mz = g.mruns[i] if i < len(g.mruns) else (np.zeros(0, np.int32),) * 2
        rec = struct.pack("<II", size, len(ns)) + np.asarray(ns, "<u4").tobytes() + \
            np.asarray(nz, "<u4").tobytes() + struct.pack("<I", len(ms)) + \
            np.asarray(ms, "<u4").tobytes() + np.asarray(mz, "<u4").tobytes() + \
            struct.pack("<I", 0) + g.packed(i).tobytes()
        index.append(struct.pack("<B", len(nm.encode())) + nm.encode() + struct.pack("<I", off))
        if off + len(rec) >= 1 << 32:
            raise ValueError("2bit v0 limited to 4 GB")
        recs.append(rec)
        off += len(rec)
    with open(path, "wb") as f:
        f.write(header)
        for x in index:
            f.write(x)
        for r in recs:
            f.write(r)


def read_sizes(path: str) -> Dict[str, int]:
    out = {}
    with open(path) as f:
        for line in f:
            w = line.split()
            if len(w) >= 2:
                out[w[0]] = int(w[1])
    return out


def write_sizes(sizes: Dict[str, int], path: str) -> None:
    with open(path, "w") as f:
        for k, v in sizes.items():
            f.write(f"{k}\t{v}\n")


# ---------------------------------------------------------------- chains
def _gap_mixture(rng, n: int, p_small: float = 0.70, p_med: float = 0.28) -> np.ndarray:
    r = rng.random(n)
    small = rng.integers(1, 30, n)
    med = np.exp(rng.uniform(np.log(30), np.log(10_000), n)).astype(np.int64)
    big = np.exp(rng.uniform(np.log(10_000), np.log(1_000_000), n)).astype(np.int64)
    return np.where(r < p_small, small, np.where(r < p_small + p_med, med, big)).astype(np.int64)


def _approx_gap_cost(dq: np.ndarray, dt: np.ndarray) -> np.ndarray:
    both = (dq > 0) & (dt > 0)
    d = np.where(both, dq + dt, np.maximum(dq, dt)).astype(float)
    q = np.interp(d, _LOOSE_POS, _LOOSE_Q, right=np.nan)
    b = np.interp(d, _LOOSE_POS, _LOOSE_B, right=np.nan)
    q = np.where(np.isnan(q), 56600 + 0.25 * (d - 252111), q)
    b = np.where(np.isnan(b), 57000 + 0.25 * (d - 252111), b)
    return np.where(both, b, q)


@dataclass
class SynthConfig:
    n_chains: int = 200_000
    alpha: float = 1.8
    max_blocks: int = 100_000
    block_mean: int = 40
    sub_rate: float = 0.12
    minus_frac: float = 0.5
    spurious_frac: float = 0.2
    max_span_frac: float = 0.5
    gap_p_small: float = 0.70   # gaps < 30 bp
    gap_p_med: float = 0.28     # 30 bp .. 10 kb (rest: 10 kb .. 1 Mb)
    seed: int = 42


def make_chains(tgen: Genome, tname: str, qgen: Genome, cfg: SynthConfig,
                mutate_query: bool = True) -> ChainArrays:
    """Plant chains target tname x all query sequences; mutates qgen in place
    (query bases under blocks := mutated target).  Returns chains sorted by
    (approximate) score, descending, ids 1..n in that order."""
    rng = np.random.default_rng(cfg.seed)
    ti = tgen.index(tname)
    tcodes = tgen.codes[ti]
    tsize = len(tcodes)
    qsizes = np.array([len(c) for c in qgen.codes], np.int64)
    n = cfg.n_chains
    spur = rng.random(n) < cfg.spurious_frac
    u = rng.random(n)
    a1 = 1.0 - cfg.alpha
    nb = np.floor((1 + u * (cfg.max_blocks ** a1 - 1)) ** (1 / a1)).astype(np.int64)
    nb = np.clip(nb, 1, cfg.max_blocks)
    nb[spur] = rng.integers(1, 6, spur.sum())
    qc = rng.choice(len(qsizes), n, p=qsizes / qsizes.sum())
    strand = (rng.random(n) < cfg.minus_frac).astype(np.uint8)
    tot = int(nb.sum())
    sizes = rng.geometric(1.0 / cfg.block_mean, tot).astype(np.int64)
    g1 = _gap_mixture(rng, tot, cfg.gap_p_small, cfg.gap_p_med)
    g2 = _gap_mixture(rng, tot, cfg.gap_p_small, cfg.gap_p_med)
    mode = rng.integers(0, 3, tot)
    dt = np.where(mode == 1, 0, g1)
    dq = np.where(mode == 0, 0, np.where(mode == 1, g1, g2))
    off = np.zeros(n + 1, np.int64)
    off[1:] = np.cumsum(nb)
    first = off[:-1]
    # last block of each chain has no gap after it
    last_idx = off[1:] - 1
    dt[last_idx] = 0
    dq[last_idx] = 0
    # truncate chains to fit max_span_frac of their sequences
    seg = np.repeat(np.arange(n), nb)
    tstep = sizes + dt
    qstep = sizes + dq
    tcum = np.cumsum(tstep) - np.repeat(np.concatenate([[0], np.cumsum(tstep)[off[1:-1] - 1]]), nb)
    qcum = np.cumsum(qstep) - np.repeat(np.concatenate([[0], np.cumsum(qstep)[off[1:-1] - 1]]), nb)
    tlim = cfg.max_span_frac * tsize
    qlim = cfg.max_span_frac * qsizes[qc][seg]
    keep = (tcum <= tlim) & (qcum <= qlim)
    keep[first] = True
    # keep must be a prefix per chain
    bad = ~keep
    firstbad = np.full(n, np.iinfo(np.int64).max)
    np.minimum.at(firstbad, seg[bad], np.nonzero(bad)[0])
    keep &= np.arange(tot) < firstbad[seg]
    sizes, dt, dq, seg = sizes[keep], dt[keep], dq[keep], seg[keep]
    nb = np.bincount(seg, minlength=n).astype(np.int64)
    off = np.zeros(n + 1, np.int64)
    off[1:] = np.cumsum(nb)
    last_idx = off[1:] - 1
    dt[last_idx] = 0
    dq[last_idx] = 0
    # clamp block sizes so that the chain fits the sequences
    size_t = np.add.reduceat(sizes + dt, off[:-1])
    size_q = np.add.reduceat(sizes + dq, off[:-1])
    ts = (rng.random(n) * (tsize - size_t)).astype(np.int64)
    qs = (rng.random(n) * (qsizes[qc] - size_q)).astype(np.int64)
    # block starts
    tstep = sizes + dt
    qstep = sizes + dq
    excl_t = np.cumsum(tstep) - tstep
    excl_q = np.cumsum(qstep) - qstep
    bt = ts[seg] + excl_t - excl_t[off[:-1]][seg]
    bq = qs[seg] + excl_q - excl_q[off[:-1]][seg]
    te = bt[last_idx] + sizes[last_idx]
    qe = bq[last_idx] + sizes[last_idx]

    # ---- plant homology & compute block scores (blastz default matrix)
    mat = matrix_by_code(_BLASTZ_ACGT)
    blk_score = np.zeros(len(sizes), np.int64)
    if mutate_query:
        order = np.argsort(qc[seg], kind="stable")
        qc_blk = qc[seg]
        for qi in np.unique(qc):
            sel = order[np.searchsorted(qc_blk[order], qi):np.searchsorted(qc_blk[order], qi, "right")]
            qcodes = qgen.codes[qi]
            qsize = len(qcodes)
            for chunk in np.array_split(sel, max(1, int(sizes[sel].sum() // 20_000_000) + 1)):
                if len(chunk) == 0:
                    continue
                lens = sizes[chunk]
                rep = np.repeat(np.arange(len(chunk)), lens)
                within = np.arange(lens.sum()) - np.repeat(np.cumsum(lens) - lens, lens)
                tpos = bt[chunk][rep] + within
                rpos = bq[chunk][rep] + within
                minus = strand[seg[chunk]][rep].astype(bool)
                tcode = tcodes[tpos]
                r = rng.random(len(tpos))
                q = tcode.copy()
                q = np.where(r < cfg.sub_rate * 2 / 3, q ^ 1, q)
                q = np.where((r >= cfg.sub_rate * 2 / 3) & (r < cfg.sub_rate * 5 / 6), q ^ 2, q)
                q = np.where((r >= cfg.sub_rate * 5 / 6) & (r < cfg.sub_rate), q ^ 3, q)
                fpos = np.where(minus, qsize - 1 - rpos, rpos)
                qcodes[fpos] = np.where(minus, q ^ 2, q).astype(np.uint8)
                blk_score[chunk] += np.bincount(rep, weights=mat[q, tcode],
                                                minlength=len(chunk)).astype(np.int64)
    gap_cost = _approx_gap_cost(dq, dt)
    gap_cost[last_idx] = 0
    score = np.add.reduceat(blk_score - gap_cost, off[:-1]).astype(np.float64)
    score = np.round(score)
    order = np.argsort(-score, kind="stable")

    tname_l = [tname] * n
    qname_l = [qgen.names[i] for i in qc]
    ca = ChainArrays(
        score=score, tname=tname_l, tsize=np.full(n, tsize, np.int32),
        tstart=ts.astype(np.int32), tend=te.astype(np.int32), qname=qname_l,
        qsize=qsizes[qc].astype(np.int32), qstrand=strand, qstart=qs.astype(np.int32),
        qend=qe.astype(np.int32), id=np.arange(1, n + 1, dtype=np.int64),
        blk_off=off, blk_t=bt.astype(np.int32), blk_q=bq.astype(np.int32),
        blk_size=sizes.astype(np.int32))
    ca = ca.subset(order)
    ca.id = np.arange(1, n + 1, dtype=np.int64)
    return ca


def small_case(seed: int = 1, n_chains: int = 300, tsize: int = 400_000,
               qsizes=(150_000, 90_000, 60_000), max_blocks: int = 400,
               n_frac: float = 0.01) -> Tuple[Genome, Genome, ChainArrays]:
    """A tiny, fast, edge-case-rich set for parity tests."""
    tg = random_genome({"chrT1": tsize}, seed, n_frac=n_frac, n_mean=200, mask_frac=0.2)
    qg = random_genome({f"chrQ{i + 1}": s for i, s in enumerate(qsizes)}, seed + 1000,
                       n_frac=n_frac, n_mean=200, mask_frac=0.2)
    cfg = SynthConfig(n_chains=n_chains, max_blocks=max_blocks, seed=seed)
    ca = make_chains(tg, "chrT1", qg, cfg)
    return tg, qg, ca


def c2_case(seed: int = 42, n_chains: int = 200_000, sizes_dir: Optional[str] = None,
            query_limit: Optional[int] = None):
    """target hg38 chr1, query all mm10 sequences."""
    here = sizes_dir or os.path.join(os.path.dirname(__file__), "data")
    hg = read_sizes(os.path.join(here, "hg38.chrom.sizes"))
    mm = read_sizes(os.path.join(here, "mm10.chrom.sizes"))
    if query_limit:
        mm = dict(list(mm.items())[:query_limit])
    tg = random_genome({"chr1": hg["chr1"]}, seed, n_frac=0.005, n_mean=20_000)
    qg = random_genome(mm, seed + 1, n_frac=0.005, n_mean=20_000)
    ca = make_chains(tg, "chr1", qg, SynthConfig(n_chains=n_chains, seed=seed))
    return tg, qg, ca


def concat_chains(parts: List[ChainArrays]) -> ChainArrays:
    """Chain sets one after another (block offsets rebased)."""
    offs, base = [np.zeros(1, np.int64)], 0
    for p in parts:
        offs.append(p.blk_off[1:] + base)
        base += int(p.blk_off[-1])
    cat = lambda k: np.concatenate([getattr(p, k) for p in parts])
    return ChainArrays(
        score=cat("score"), tname=[x for p in parts for x in p.tname], tsize=cat("tsize"),
        tstart=cat("tstart"), tend=cat("tend"), qname=[x for p in parts for x in p.qname],
        qsize=cat("qsize"), qstrand=cat("qstrand"), qstart=cat("qstart"), qend=cat("qend"),
        id=cat("id"), blk_off=np.concatenate(offs), blk_t=cat("blk_t"), blk_q=cat("blk_q"),
        blk_size=cat("blk_size"))


def c5_case(seed: int = 1234, n_chains: int = 1_000_000, sizes_dir: Optional[str] = None,
            scale: float = 1.0, min_size: int = 20_000):
    """SURVEY §8(d) C5 at a stated chain count: every hg38 sequence (455) as
    target x every mm10 sequence (66) as query, chains per target sequence in
    proportion to its length, C2's chain model on each; one score-sorted set
    (ids 1..n).  scale < 1 shrinks every sequence (not below min_size) for
    C5-shaped parity tests: same names, same sequence count."""
    here = sizes_dir or os.path.join(os.path.dirname(__file__), "data")
    hg = read_sizes(os.path.join(here, "hg38.chrom.sizes"))
    mm = read_sizes(os.path.join(here, "mm10.chrom.sizes"))
    if scale != 1.0:
        hg = {k: max(min_size, int(v * scale)) for k, v in hg.items()}
        mm = {k: max(min_size, int(v * scale)) for k, v in mm.items()}
    tg = random_genome(hg, seed, n_frac=0.005, n_mean=20_000)
    qg = random_genome(mm, seed + 1, n_frac=0.005, n_mean=20_000)
    total = float(sum(hg.values()))
    parts = []
    for k, (name, size) in enumerate(hg.items()):
        nc = int(round(n_chains * size / total))
        if nc > 0:
            parts.append(make_chains(tg, name, qg, SynthConfig(n_chains=nc, seed=seed + 7 * (k + 1))))
    ca = concat_chains(parts)
    ca = ca.subset(np.argsort(-ca.score, kind="stable"))
    ca.id = np.arange(1, ca.n + 1, dtype=np.int64)
    return tg, qg, ca


def zero_end_blocks(ca: ChainArrays, every: int = 3) -> ChainArrays:
    """Every `every`-th chain gets a zero-size block 3/2 bases before its
    first block and 4/1 bases after its last (header span widened)."""
    bt, bq, bs, off = [], [], [], [0]
    tstart, tend = ca.tstart.copy(), ca.tend.copy()
    qstart, qend = ca.qstart.copy(), ca.qend.copy()
    for i in range(ca.n):
        t, q, z = (x.astype(np.int64) for x in ca.blocks(i))
        if i % every == 0 and t[0] >= 3 and q[0] >= 2 and \
                t[-1] + z[-1] + 4 <= ca.tsize[i] and q[-1] + z[-1] + 1 <= ca.qsize[i]:
            t = np.r_[t[0] - 3, t, t[-1] + z[-1] + 4]
            q = np.r_[q[0] - 2, q, q[-1] + z[-1] + 1]
            z = np.r_[0, z, 0]
            tstart[i], qstart[i] = t[0], q[0]
            tend[i], qend[i] = t[-1], q[-1]
        bt.append(t)
        bq.append(q)
        bs.append(z)
        off.append(off[-1] + len(t))
    return ChainArrays(score=ca.score, tname=ca.tname, tsize=ca.tsize, tstart=tstart, tend=tend,
                       qname=ca.qname, qsize=ca.qsize, qstrand=ca.qstrand, qstart=qstart,
                       qend=qend, id=ca.id, blk_off=np.asarray(off, np.int64),
                       blk_t=np.concatenate(bt).astype(np.int32),
                       blk_q=np.concatenate(bq).astype(np.int32),
                       blk_size=np.concatenate(bs).astype(np.int32))


# ---------------------------------------------------------------- chainCleaner loci
def _mutate(rng, codes: np.ndarray, div: float) -> np.ndarray:
    r = rng.random(len(codes))
    q = codes.copy()
    q = np.where(r < div * 2 / 3, q ^ 1, q)
    q = np.where((r >= div * 2 / 3) & (r < div * 5 / 6), q ^ 2, q)
    q = np.where((r >= div * 5 / 6) & (r < div), q ^ 3, q)
    return q.astype(np.uint8)


class _Chain:
    def __init__(self, tname: str, qname: str, strand: int):
        self.tname, self.qname, self.strand = tname, qname, strand
        self.blocks: List[Tuple[int, int, int, float]] = []  # (t, q, size, div)

    def add_run(self, rng, t: int, q: int, length: int, div: float, bmin=80, bmax=600,
                gmax=40) -> Tuple[int, int]:
        """Blocks covering about `length` target bases from (t, q) with small
        gaps (one- or two-sided); returns the end (t, q)."""
        end = t + length
        while True:
            size = int(rng.integers(bmin, bmax + 1))
            if t + size >= end:
                size = max(1, end - t)
                self.blocks.append((t, q, size, div))
                return t + size, q + size
            self.blocks.append((t, q, size, div))
            t += size
            q += size
            mode = int(rng.integers(0, 3))
            g1, g2 = int(rng.integers(1, gmax + 1)), int(rng.integers(1, gmax + 1))
            t += 0 if mode == 1 else g1
            q += 0 if mode == 0 else g2
            if t >= end - 10:
                return t, q


def cleaner_case(seed: int = 7, n_loci: int = 24, genomes=None, tmap=None, qmap=None,
                 t_origin=None, q_origin=None):
    """Planted chain-breaking alignments (chainCleaner).

    Per locus a high-scoring chain P (the would-be breaking chain) has two
    long anchors and, between them, 1-3 short "suspect" runs separated by
    large gaps; a lower-scoring chain B aligns a different query region to
    the target inside those gaps, so in the nets B is split by P's suspects
    (1-3 breaks, adjacent pairs for -doPairs).  Suspect size/divergence and
    B's piece sizes/divergence are drawn so that some suspects pass the
    default thresholds and others fail one (LR ratio, broken-chain score,
    gap size); extra chains sometimes sit between B's pieces (breaks that
    stay broken by another higher-scoring chain), B is on either strand, and
    unrelated noise chains (with exact score ties) fill the space between
    loci.  Header scores are left 0: the caller rescores the chains with the
    reference scoreChain, sorts them and assigns ids.
    genomes=(tg, qg) plants the loci into existing genomes instead (the
    chr1-scale C3 set): tmap/qmap map the logical names chrT1/chrT2 and
    chrQ1..3 to sequences of those genomes, t_origin/q_origin give the first
    target position of each logical target and the first query position of
    each logical query (their regions must not overlap).
    Returns (target Genome, query Genome, list of _Chain)."""
    rng = np.random.default_rng(seed)
    span = 56_000
    tsizes = {"chrT1": (n_loci // 2 + 1) * span + 20_000,
              "chrT2": (n_loci - n_loci // 2 + 1) * span + 20_000}
    qsizes = {"chrQ1": sum(tsizes.values()) + 40_000, "chrQ2": n_loci * 36_000 + 20_000,
              "chrQ3": n_loci * 30_000 + 20_000}
    if genomes is None:
        tg = random_genome(tsizes, seed, n_frac=0.0)
        qg = random_genome(qsizes, seed + 1, n_frac=0.0)
        tmap = {k: k for k in tsizes}
        qmap = {k: k for k in qsizes}
        t_origin = {"chrT1": 5_000, "chrT2": 5_000}
        q_origin = {"chrQ1": 1000, "chrQ2": 1000, "chrQ3": 1000}
    else:
        tg, qg = genomes
        full = qg.sizes
        for k in qsizes:  # the logical query's region ends where its sequence does
            qsizes[k] = full[qmap[k]]
            assert q_origin[k] + {"chrQ1": sum(tsizes.values()) + 40_000,
                                  "chrQ2": n_loci * 36_000 + 20_000,
                                  "chrQ3": n_loci * 30_000 + 20_000}[k] < qsizes[k], k
    chains: List[_Chain] = []
    qcur = dict(q_origin)  # forward allocation cursors

    def q_alloc(qname: str, length: int, strand: int) -> int:
        """Allocate `length` forward bases; return the start in strand coords."""
        f = qcur[qname]
        qcur[qname] = f + length + int(rng.integers(200, 2000))
        assert qcur[qname] < qsizes[qname], qname
        return f if strand == 0 else qsizes[qname] - (f + length)

    def chain(tname: str, qname: str, strand: int) -> "_Chain":
        return _Chain(tmap[tname], qmap[qname], strand)

    locus_t = dict(t_origin)
    for li in range(n_loci):
        tname = "chrT1" if li % 2 == 0 else "chrT2"
        x = locus_t[tname]
        locus_t[tname] += span
        # every 4th locus: two strong suspects around a tiny divergent middle
        # piece of B -- both singles fail on that side, the pair can pass
        pair_locus = li % 4 == 3
        k = 2 if pair_locus else int(rng.choice([1, 1, 2, 2, 3]))
        a_lo, a_hi = (8000, 10000) if pair_locus else (2500, 5000)
        a_l, a_r = int(rng.integers(a_lo, a_hi)), int(rng.integers(a_lo, a_hi))
        gaps = [int(rng.integers(6000, 11000)) for _ in range(k + 1)]
        susp = [int(rng.choice([150, 250] if pair_locus else [20, 40, 80, 150, 300, 700]))
                for _ in range(k)]
        # ---- P on chrQ1 '+': anchors, gaps (two-sided), suspects
        p = chain(tname, "chrQ1", 0)
        total_t = a_l + sum(gaps) + sum(susp) + a_r
        q0 = q_alloc("chrQ1", total_t + 600 * (k + 1), 0)
        t, q = p.add_run(rng, x, q0, a_l, 0.04)
        gap_iv, susp_iv = [], []
        for j in range(k + 1):
            g_t = gaps[j]
            g_q = max(50, g_t + int(rng.integers(-400, 400)))
            gap_iv.append((t, t + g_t))
            t += g_t
            q += g_q
            if j < k:
                sdiv = 0.05 if pair_locus else float(rng.choice([0.05, 0.15, 0.25, 0.35]))
                s0 = t
                t, q = p.add_run(rng, t, q, susp[j], sdiv, bmin=20, bmax=400, gmax=30)
                susp_iv.append((s0, t))
        t, q = p.add_run(rng, t, q, a_r, 0.04)
        chains.append(p)
        # ---- B: one piece per P gap, on chrQ2 either strand
        strand = int(rng.integers(0, 2))
        bdiv = 0.06 if pair_locus else float(rng.choice([0.06, 0.1, 0.14, 0.3]))
        pieces = []
        for (g0, g1) in gap_iv:
            glen = g1 - g0
            m1 = int(rng.integers(100, glen // 3))
            m2 = int(rng.integers(100, glen // 3))
            inner = 0 < len(pieces) < len(gap_iv) - 1
            if pair_locus:
                length = 120 if inner else min(2500, glen - m1 - m2 - 50)
            else:
                length = int(rng.choice([120, 200, 400] if inner and rng.random() < 0.5 else
                                        [300, 800, 1500, 2500, glen - m1 - m2 - 50]))
            length = max(100, min(length, glen - m1 - m2 - 50))
            # the piece hugs the suspect side of the gap
            pieces.append((g0 + m1, g0 + m1 + length) if len(pieces) == len(gap_iv) - 1
                          else (g1 - m2 - length, g1 - m2))
        # first piece sits at the right end of the first gap (next to the
        # suspect), the last at the left end of the last gap
        qlen = sum(b - a for a, b in pieces) + 400 * len(pieces) + 5000
        bq = q_alloc("chrQ2", qlen, strand)
        b = chain(tname, "chrQ2", strand)
        qb = bq
        for pi, (a0, a1) in enumerate(pieces):
            tiny = pair_locus and 0 < pi < len(pieces) - 1
            _, qb = b.add_run(rng, a0, qb, a1 - a0, 0.3 if tiny else bdiv)
            qb += int(rng.integers(5, 300))
        chains.append(b)
        # ---- sometimes a third chain inside a gap, next to one of B's pieces
        if rng.random() < 0.3:
            j = int(rng.integers(0, len(gap_iv)))
            g0, g1 = gap_iv[j]
            a0, a1 = pieces[j]
            lo, hi = (g0 + 20, a0 - 20) if a0 - g0 > g1 - a1 else (a1 + 20, g1 - 20)
            if hi - lo > 200:
                c = chain(tname, "chrQ3", int(rng.integers(0, 2)))
                clen = int(rng.integers(150, hi - lo))
                c0 = int(rng.integers(lo, hi - clen + 1))
                cq = q_alloc("chrQ3", clen + 200, c.strand)
                c.add_run(rng, c0, cq, clen, float(rng.choice([0.02, 0.1, 0.2])))
                chains.append(c)
        # ---- noise chains in the spacer after the locus
        t_sp = x + total_t + 200
        n_noise = 0
        while t_sp + 900 < x + span - 200 and n_noise < 10:
            n_noise += 1
            n_len = int(rng.integers(60, 700))
            c = chain(tname, "chrQ3", int(rng.integers(0, 2)))
            cq = q_alloc("chrQ3", n_len + 100, c.strand)
            c.add_run(rng, t_sp, cq, n_len, float(rng.choice([0.0, 0.1, 0.3])), bmin=30,
                      bmax=300)
            chains.append(c)
            t_sp += n_len + int(rng.integers(50, 800))
    # ---- plant homology
    for c in chains:
        ti, qi = tg.index(c.tname), qg.index(c.qname)
        qcodes = qg.codes[qi]
        qsize = len(qcodes)
        for (t, q, size, div) in c.blocks:
            m = _mutate(rng, tg.codes[ti][t:t + size], div)
            if c.strand == 0:
                qcodes[q:q + size] = m
            else:
                f0 = qsize - (q + size)
                qcodes[f0:f0 + size] = (m ^ 2)[::-1]
    # ---- exact score ties: duplicate a few noise chains' target and query text
    noise = [c for c in chains
             if c.qname == qmap["chrQ3"] and len(c.blocks) == 1 and c.blocks[0][3] == 0.0]
    for a, b2 in zip(noise[0::2], noise[1::2]):
        (ta, qa, sa, _), (tb, qb, sb, _) = a.blocks[0], b2.blocks[0]
        s = min(sa, sb)
        a.blocks[0] = (ta, qa, s, 0.0)
        b2.blocks[0] = (tb, qb, s, 0.0)
        ti = tg.index(a.tname)
        tg.codes[tg.index(b2.tname)][tb:tb + s] = tg.codes[ti][ta:ta + s]
        for c in (a, b2):
            t, q, size, _ = c.blocks[0]
            qcodes = qg.codes[qg.index(c.qname)]
            m = tg.codes[tg.index(c.tname)][t:t + size]
            if c.strand == 0:
                qcodes[q:q + size] = m
            else:
                f0 = len(qcodes) - (q + size)
                qcodes[f0:f0 + size] = (m ^ 2)[::-1]
    return tg, qg, chains


def c3_case(seed: int = 42, n_chains: int = 200_000, n_loci: int = 1000,
            sizes_dir: Optional[str] = None):
    """C2 (hg38 chr1 x all mm10, n_chains background chains)
    plus n_loci planted chain-breaking-alignment loci (cleaner_case's loci:
    a higher-scoring chain whose short suspect runs break a lower chain into
    pieces) in chr1 30 Mb onwards, their query sides on mm10 chr1/chr2/chr3.
    The loci's header scores are 0 and the background's approximate: the
    caller rescores every chain (scoreChain), sorts by score and numbers
    them, as the reference pipeline would have."""
    tg, qg, bg = c2_case(seed, n_chains, sizes_dir)
    span = 56_000
    t1 = 30_000_000
    t2 = t1 + (n_loci // 2 + 1) * span + 120_000
    _, _, loci = cleaner_case(seed + 1, n_loci, genomes=(tg, qg),
                              tmap={"chrT1": "chr1", "chrT2": "chr1"},
                              qmap={"chrQ1": "chr1", "chrQ2": "chr2", "chrQ3": "chr3"},
                              t_origin={"chrT1": t1, "chrT2": t2},
                              q_origin={"chrQ1": 1_000_000, "chrQ2": 1_000_000, "chrQ3": 1_000_000})
    return tg, qg, concat_chains([bg, chains_to_arrays(tg, qg, loci)])


def chains_to_arrays(tg: Genome, qg: Genome, chains) -> ChainArrays:
    """_Chain list -> ChainArrays (score 0, ids 1..n in list order)."""
    n = len(chains)
    offs = [0]
    bt, bq, bs = [], [], []
    ts, te, qs, qe = [], [], [], []
    for c in chains:
        for (t, q, s, _) in c.blocks:
            bt.append(t)
            bq.append(q)
            bs.append(s)
        offs.append(len(bs))
        ts.append(c.blocks[0][0])
        qs.append(c.blocks[0][1])
        te.append(c.blocks[-1][0] + c.blocks[-1][2])
        qe.append(c.blocks[-1][1] + c.blocks[-1][2])
    tsz, qsz = tg.sizes, qg.sizes
    return ChainArrays(
        score=np.zeros(n), tname=[c.tname for c in chains],
        tsize=np.array([tsz[c.tname] for c in chains], np.int32),
        tstart=np.array(ts, np.int32), tend=np.array(te, np.int32),
        qname=[c.qname for c in chains], qsize=np.array([qsz[c.qname] for c in chains], np.int32),
        qstrand=np.array([c.strand for c in chains], np.uint8), qstart=np.array(qs, np.int32),
        qend=np.array(qe, np.int32), id=np.arange(1, n + 1, dtype=np.int64),
        blk_off=np.array(offs, np.int64), blk_t=np.array(bt, np.int32),
        blk_q=np.array(bq, np.int32), blk_size=np.array(bs, np.int32))


# ---------------------------------------------------------------- axtChain PSL input
def psl_case(seed: int = 5, tsizes=(300_000, 120_000), qsizes=(250_000, 90_000),
             paths_per_pair: int = 6, noise_frac: float = 0.2):
    """Seeded PSL blocks for axtChain (small): per
    (target, query, strand) pair a few planted collinear alignment paths --
    ungapped blocks (geometric sizes) separated by q/t/both gaps, query bases a
    mutated copy of the target -- cut into PSL records of 1-8 blocks; then
    the awkward cases the DP has to get right: records re-emitted with a
    diagonal shift (partially overlapping blocks -> crossovers), records
    re-emitted from the same start with another length (removeExactOverlaps
    folds), blocks overlapping the previous block on one side only, and
    random unrelated blocks (noise_frac).  Both strands; N runs in both
    genomes.  Returns (target Genome, query Genome, list of PSL records as
    (qName, strand, tName, [(tStart, qStart, size)...]))."""
    rng = np.random.default_rng(seed)
    tg = random_genome({f"chrT{i + 1}": s for i, s in enumerate(tsizes)}, seed, n_frac=0.002,
                       n_mean=300)
    qg = random_genome({f"chrQ{i + 1}": s for i, s in enumerate(qsizes)}, seed + 1, n_frac=0.002,
                       n_mean=300)
    recs = []
    for ti, tname in enumerate(tg.names):
        tcodes = tg.codes[ti]
        for qi, qname in enumerate(qg.names):
            qcodes = qg.codes[qi]
            qsize = len(qcodes)
            for strand in (0, 1):
                sname = "+-"[strand]
                for _ in range(paths_per_pair):
                    nblk = int(rng.integers(3, 60))
                    t = int(rng.integers(0, len(tcodes) // 2))
                    q = int(rng.integers(0, qsize // 2))
                    div = float(rng.choice([0.05, 0.12, 0.2]))
                    path = []
                    for _b in range(nblk):
                        size = int(min(rng.geometric(1 / 60), 400))
                        if t + size >= len(tcodes) or q + size >= qsize:
                            break
                        path.append((t, q, size))
                        m = _mutate(rng, tcodes[t:t + size], div)
                        if strand == 0:
                            qcodes[q:q + size] = m
                        else:
                            f0 = qsize - (q + size)
                            qcodes[f0:f0 + size] = (m ^ 2)[::-1]
                        mode = int(rng.integers(0, 3))
                        g = int(rng.choice([1, 3, 10, 40, 200, 1500, 8000]))
                        t += size + (0 if mode == 1 else g)
                        q += size + (0 if mode == 0 else int(rng.integers(1, 2 * g + 2)))
                    # cut into records
                    i = 0
                    while i < len(path):
                        k = int(rng.integers(1, 9))
                        rec = path[i:i + k]
                        recs.append((qname, sname, tname, list(rec)))
                        r = rng.random()
                        if r < 0.15:     # diagonal shift: partial overlaps
                            d = int(rng.integers(1, 25))
                            shifted = [(a + d, b + d, s) for a, b, s in rec
                                       if a + d + s < len(tcodes) and b + d + s < qsize]
                            if shifted:
                                recs.append((qname, sname, tname, shifted))
                        elif r < 0.25:   # same starts, other length
                            recs.append((qname, sname, tname,
                                         [(a, b, max(1, s + int(rng.integers(-20, 20))))
                                          for a, b, s in rec]))
                        elif r < 0.32:   # one-sided overlap with the previous block
                            a, b, s = rec[0]
                            if s > 30:
                                recs.append((qname, sname, tname, [(a + 10, b + 5, s - 15)]))
                        i += k
                # noise blocks
                nn = int(noise_frac * paths_per_pair * 20)
                for _ in range(nn):
                    size = int(rng.integers(20, 200))
                    t = int(rng.integers(0, len(tcodes) - size))
                    q = int(rng.integers(0, qsize - size))
                    recs.append((qname, sname, tname, [(t, q, size)]))
    order = rng.permutation(len(recs))
    return tg, qg, [recs[i] for i in order]


def write_psl(tg: Genome, qg: Genome, recs, path: str, header: bool = True) -> None:
    """PSL text (psLayout version 3): only strand, names, sizes and the
    block lists matter to axtChain; match counts are left 0."""
    tsz, qsz = tg.sizes, qg.sizes
    with open(path, "w") as f:
        if header:
            f.write("psLayout version 3\n\nmatch\tmis-\trep.\tN's\tQ gap\tQ gap\tT gap\tT gap\t"
                    "strand\tQ\t\tQ\tQ\tQ\tT\t\tT\tT\tT\tblock\tblockSizes\tqStarts\t tStarts\n"
                    "\tmatch\tmatch\t\tcount\tbases\tcount\tbases\t\tname\t\tsize\tstart\tend\t"
                    "name\t\tsize\tstart\tend\tcount\n" + "-" * 159 + "\n")
        for qname, strand, tname, blocks in recs:
            blocks = sorted(blocks, key=lambda b: (b[0], b[1]))
            ts = blocks[0][0]
            te = max(a + s for a, b, s in blocks)
            qs = min(b for a, b, s in blocks)
            qe = max(b + s for a, b, s in blocks)
            if strand == "-":
                qs, qe = qsz[qname] - qe, qsz[qname] - qs
            f.write("\t".join(str(x) for x in [0, 0, 0, 0, 0, 0, 0, 0, strand, qname, qsz[qname], qs,
                                                qe, tname, tsz[tname], ts, te, len(blocks)]))
            f.write("\t" + "".join(f"{s}," for a, b, s in blocks))
            f.write("\t" + "".join(f"{b}," for a, b, s in blocks))
            f.write("\t" + "".join(f"{a}," for a, b, s in blocks) + "\n")


def psl_c4(seed: int = 7, n_blocks: int = 2_000_000, n_t: int = 4, n_q: int = 3,
           tsize: int = 60_000_000, qsize: int = 50_000_000, collinear: float = 0.8,
           alpha: float = 1.2):
    """SURVEY §8(d) C4 at a chosen size: n_blocks PSL blocks over n_t x n_q
    chromosome pairs x 2 strands, power-law blocks per pair, `collinear` of
    them on planted collinear paths (mutated copies, gaps mostly short) and
    the rest random.  Vectorised; returns (tg, qg, recs-as-arrays) where
    recs = dict(pair arrays: qname, strand, tname; per-block arrays:
    rec (record id), t, q, size; per-record pair index)."""
    rng = np.random.default_rng(seed)
    tg = random_genome({f"chr{i + 1}": tsize for i in range(n_t)}, seed, n_frac=0.001,
                       n_mean=2000)
    qg = random_genome({f"chrQ{i + 1}": qsize for i in range(n_q)}, seed + 1, n_frac=0.001,
                       n_mean=2000)
    pairs = [(ti, qi, s) for ti in range(n_t) for qi in range(n_q) for s in (0, 1)]
    w = 1.0 / np.arange(1, len(pairs) + 1) ** alpha
    w = w[rng.permutation(len(pairs))]
    per_pair = np.maximum(50, (w / w.sum() * n_blocks).astype(np.int64))
    out_t, out_q, out_s, out_pair, out_rec = [], [], [], [], []
    rec_base = 0
    mat = matrix_by_code(_BLASTZ_ACGT)
    for pi, (ti, qi, strand) in enumerate(pairs):
        nb = int(per_pair[pi])
        ncol = int(nb * collinear)
        # collinear paths of ~200 blocks each
        npath = max(1, ncol // 200)
        sizes = np.minimum(rng.geometric(1 / 50, ncol), 500).astype(np.int64)
        mode = rng.integers(0, 3, ncol)
        g = np.where(rng.random(ncol) < 0.8, rng.integers(1, 60, ncol),
                     rng.integers(60, 5000, ncol))
        dt = np.where(mode == 1, 0, g)
        dq = np.where(mode == 0, 0, np.maximum(1, g + rng.integers(-20, 20, ncol)))
        path = np.minimum(np.arange(ncol) * npath // max(ncol, 1), npath - 1)
        first = np.r_[True, path[1:] != path[:-1]]
        tstep = np.where(first, 0, np.r_[0, (sizes + dt)[:-1]])
        qstep = np.where(first, 0, np.r_[0, (sizes + dq)[:-1]])
        # path origins
        span_t = np.bincount(path, weights=sizes + dt, minlength=npath)
        span_q = np.bincount(path, weights=sizes + dq, minlength=npath)
        t0 = (rng.random(npath) * np.maximum(1, tsize - span_t - 1)).astype(np.int64)
        q0 = (rng.random(npath) * np.maximum(1, qsize - span_q - 1)).astype(np.int64)
        ct = np.cumsum(tstep) - np.repeat(np.cumsum(tstep)[first], np.bincount(path))
        cq = np.cumsum(qstep) - np.repeat(np.cumsum(qstep)[first], np.bincount(path))
        bt = t0[path] + ct
        bq = q0[path] + cq
        ok = (bt + sizes < tsize) & (bq + sizes < qsize)
        bt, bq, sizes, path = bt[ok], bq[ok], sizes[ok], path[ok]
        # plant homology (12% substitutions)
        tc = tg.codes[ti]
        qc = qg.codes[qi]
        rep = np.repeat(np.arange(len(sizes)), sizes)
        within = np.arange(sizes.sum()) - np.repeat(np.cumsum(sizes) - sizes, sizes)
        tpos = bt[rep] + within
        rpos = bq[rep] + within
        m = _mutate(rng, tc[tpos], 0.12)
        fpos = rpos if strand == 0 else qsize - 1 - rpos
        qc[fpos] = m if strand == 0 else m ^ 2
        # random blocks
        nr = nb - ncol
        rs = rng.integers(20, 300, nr)
        rt = rng.integers(0, tsize - 400, nr)
        rq = rng.integers(0, qsize - 400, nr)
        # records: collinear blocks in runs of 1..8 consecutive blocks
        k = rng.integers(1, 9, len(sizes))
        rec_c = np.cumsum(np.r_[0, (np.arange(1, len(sizes)) % 5 == 0) |
                                (path[1:] != path[:-1])]) if len(sizes) else np.zeros(0, np.int64)
        del k
        rec_r = np.arange(nr) + (rec_c[-1] + 1 if len(rec_c) else 0)
        out_t += [bt, rt]
        out_q += [bq, rq]
        out_s += [sizes, rs]
        out_pair += [np.full(len(sizes) + nr, pi, np.int32)]
        out_rec += [rec_base + rec_c, rec_base + rec_r]
        rec_base += int((rec_r[-1] + 1) if nr else (rec_c[-1] + 1 if len(rec_c) else 0))
    blocks = dict(t=np.concatenate(out_t).astype(np.int64), q=np.concatenate(out_q).astype(np.int64),
                  size=np.concatenate(out_s).astype(np.int64),
                  pair=np.concatenate(out_pair), rec=np.concatenate(out_rec).astype(np.int64))
    return tg, qg, pairs, blocks


def write_psl_c4(tg: Genome, qg: Genome, pairs, blocks, path: str, seed: int = 7) -> int:
    """PSL text of psl_c4 blocks: one line per record, records in a seeded
    random order (as lastz output of many jobs would be concatenated)."""
    rng = np.random.default_rng(seed + 99)
    rec = blocks["rec"]
    order = np.argsort(rec, kind="stable")
    rec_s = rec[order]
    starts = np.r_[0, np.nonzero(rec_s[1:] != rec_s[:-1])[0] + 1]
    ends = np.r_[starts[1:], len(rec_s)]
    perm = rng.permutation(len(starts))
    tnames = tg.names
    qnames = qg.names
    tsz = tg.sizes
    qsz = qg.sizes
    with open(path, "w") as f:
        for r in perm:
            idx = order[starts[r]:ends[r]]
            pi = int(blocks["pair"][idx[0]])
            ti, qi, strand = pairs[pi]
            bt = blocks["t"][idx]
            bq = blocks["q"][idx]
            bs = blocks["size"][idx]
            o = np.lexsort((bq, bt))
            bt, bq, bs = bt[o], bq[o], bs[o]
            tn, qn = tnames[ti], qnames[qi]
            qs, qe = int(bq.min()), int((bq + bs).max())
            if strand:
                qs, qe = qsz[qn] - qe, qsz[qn] - qs
            f.write(f"0\t0\t0\t0\t0\t0\t0\t0\t{'+-'[strand]}\t{qn}\t{qsz[qn]}\t{qs}\t{qe}\t{tn}\t"
                    f"{tsz[tn]}\t{int(bt[0])}\t{int((bt + bs).max())}\t{len(bt)}\t"
                    + "".join(f"{x}," for x in bs) + "\t" + "".join(f"{x}," for x in bq)
                    + "\t" + "".join(f"{x}," for x in bt) + "\n")
    return len(starts)
