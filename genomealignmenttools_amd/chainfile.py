"""Host-side .chain reader/writer (struct-of-arrays), Python mirror of
kent/src/lib/chain.c:200-346 (chainWriteHead/chainWrite/chainReadChainLine/
chainReadBlocks).  Used by tests, the synthetic generators and bench.py; the
C tools in csrc/tools have their own streaming parser.
"""
from __future__ import annotations

import gzip
import io
from dataclasses import dataclass, field
from typing import List, Optional

import numpy as np


@dataclass
class ChainArrays:
    score: np.ndarray          # float64 header score
    tname: List[str]
    tsize: np.ndarray          # int32
    tstart: np.ndarray
    tend: np.ndarray
    qname: List[str]
    qsize: np.ndarray
    qstrand: np.ndarray        # uint8 0 '+', 1 '-'
    qstart: np.ndarray
    qend: np.ndarray
    id: np.ndarray             # int64
    blk_off: np.ndarray        # int64 [n+1]
    blk_t: np.ndarray          # int32 tStart of each block
    blk_q: np.ndarray          # int32 qStart (chain strand coordinates)
    blk_size: np.ndarray       # int32
    meta: List[str] = field(default_factory=list)  # '#' lines

    @property
    def n(self) -> int:
        return len(self.tname)

    def blocks(self, i: int):
        a, b = int(self.blk_off[i]), int(self.blk_off[i + 1])
        return self.blk_t[a:b], self.blk_q[a:b], self.blk_size[a:b]

    def aligned_bases(self) -> int:
        return int(self.blk_size.sum(dtype=np.int64))

    def subset(self, idx) -> "ChainArrays":
        idx = np.asarray(idx, dtype=np.int64)
        offs = [0]
        bt, bq, bs = [], [], []
        for i in idx:
            t, q, s = self.blocks(int(i))
            bt.append(t)
            bq.append(q)
            bs.append(s)
            offs.append(offs[-1] + len(s))
        cat = (lambda xs: np.concatenate(xs).astype(np.int32) if xs else np.zeros(0, np.int32))
        return ChainArrays(
            score=self.score[idx], tname=[self.tname[i] for i in idx], tsize=self.tsize[idx],
            tstart=self.tstart[idx], tend=self.tend[idx], qname=[self.qname[i] for i in idx],
            qsize=self.qsize[idx], qstrand=self.qstrand[idx], qstart=self.qstart[idx],
            qend=self.qend[idx], id=self.id[idx], blk_off=np.asarray(offs, np.int64),
            blk_t=cat(bt), blk_q=cat(bq), blk_size=cat(bs), meta=list(self.meta))


def _open_text(path: str) -> str:
    if path == "stdin":
        import sys
        return sys.stdin.read()
    with open(path, "rb") as f:
        raw = f.read()
    if raw[:2] == b"\x1f\x8b":
        raw = gzip.decompress(raw)
    return raw.decode()


def read_chains(path: str) -> ChainArrays:
    """Parse a .chain file.  Missing ids get 1, 2, ... like chainIdNext."""
    text = _open_text(path)
    score, tname, tsize, tstart, tend = [], [], [], [], []
    qname, qsize, qstrand, qstart, qend, ids = [], [], [], [], [], []
    offs = [0]
    bt, bq, bs = [], [], []
    meta = []
    next_id = 1
    lines = text.split("\n")
    i, n = 0, len(lines)
    while i < n:
        line = lines[i]
        i += 1
        if line.startswith("#"):
            meta.append(line)
            continue
        w = line.split()
        if not w:
            continue
        if w[0] != "chain" or len(w) < 12:
            raise ValueError(f"Expecting 'chain' line {i} of {path}")
        score.append(float(w[1]))
        tname.append(w[2])
        tsize.append(int(w[3]))
        ts, te = int(w[5]), int(w[6])
        qname.append(w[7])
        qsize.append(int(w[8]))
        qstrand.append(1 if w[9][0] == "-" else 0)
        qs, qe = int(w[10]), int(w[11])
        if len(w) >= 13:
            ids.append(int(w[12]))
        else:
            ids.append(next_id)
            next_id += 1
        tstart.append(ts)
        tend.append(te)
        qstart.append(qs)
        qend.append(qe)
        t, q = ts, qs
        while True:
            if i >= n:
                raise ValueError(f"unexpected end of {path}")
            bl = lines[i]
            i += 1
            if bl.startswith("#"):
                meta.append(bl)
                continue
            bw = bl.split()
            if not bw:
                continue
            size = int(bw[0])
            bt.append(t)
            bq.append(q)
            bs.append(size)
            t += size
            q += size
            if len(bw) == 1:
                break
            if len(bw) < 3:
                raise ValueError(f"Expecting 1 or 3 words line {i} of {path}")
            t += int(bw[1])
            q += int(bw[2])
        if q != qe or t != te:
            raise ValueError(f"end mismatch in chain ending line {i} of {path}")
        offs.append(len(bs))
    as32 = lambda x: np.asarray(x, dtype=np.int32)
    return ChainArrays(
        score=np.asarray(score, np.float64), tname=tname, tsize=as32(tsize),
        tstart=as32(tstart), tend=as32(tend), qname=qname, qsize=as32(qsize),
        qstrand=np.asarray(qstrand, np.uint8), qstart=as32(qstart), qend=as32(qend),
        id=np.asarray(ids, np.int64), blk_off=np.asarray(offs, np.int64), blk_t=as32(bt),
        blk_q=as32(bq), blk_size=as32(bs), meta=meta)


def fmt_score(x: float) -> str:
    """C printf("%1.0f") (round-half-even of the double)."""
    return "%1.0f" % x


def write_chains(ca: ChainArrays, path_or_file, scores: Optional[np.ndarray] = None) -> None:
    """chainWrite (kent/src/lib/chain.c:200-227) for every chain."""
    own = isinstance(path_or_file, str)
    f = open(path_or_file, "w") if own else path_or_file
    try:
        buf = io.StringIO()
        sc = ca.score if scores is None else scores
        for i in range(ca.n):
            buf.write("chain %s %s %d + %d %d %s %d %s %d %d %d\n" % (
                fmt_score(sc[i]), ca.tname[i], ca.tsize[i], ca.tstart[i], ca.tend[i],
                ca.qname[i], ca.qsize[i], "-" if ca.qstrand[i] else "+", ca.qstart[i],
                ca.qend[i], ca.id[i]))
            t, q, s = ca.blocks(i)
            m = len(s)
            if m > 1:
                dt = t[1:] - (t[:-1] + s[:-1])
                dq = q[1:] - (q[:-1] + s[:-1])
                body = "\n".join("%d\t%d\t%d" % v for v in zip(s[:-1], dt, dq))
                buf.write(body + "\n")
            buf.write("%d\n\n" % s[-1])
            if buf.tell() > (1 << 22):
                f.write(buf.getvalue())
                buf = io.StringIO()
        f.write(buf.getvalue())
    finally:
        if own:
            f.close()
