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
        lens = self.blk_off[idx + 1] - self.blk_off[idx]
        offs = np.zeros(len(idx) + 1, np.int64)
        np.cumsum(lens, out=offs[1:])
        src = np.repeat(self.blk_off[idx] - offs[:-1], lens) + np.arange(offs[-1], dtype=np.int64)
        as32 = lambda x: np.ascontiguousarray(x[src], dtype=np.int32)
        return ChainArrays(
            score=self.score[idx], tname=[self.tname[i] for i in idx], tsize=self.tsize[idx],
            tstart=self.tstart[idx], tend=self.tend[idx], qname=[self.qname[i] for i in idx],
            qsize=self.qsize[idx], qstrand=self.qstrand[idx], qstart=self.qstart[idx],
            qend=self.qend[idx], id=self.id[idx], blk_off=offs,
            blk_t=as32(self.blk_t), blk_q=as32(self.blk_q), blk_size=as32(self.blk_size),
            meta=list(self.meta))


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


# ---------------------------------------------------------------- fast writer
def _ndig(v: np.ndarray) -> np.ndarray:
    """Decimal digits of |v| (int64), sign excluded."""
    a = np.abs(v)
    nd = np.ones(len(a), np.int64)
    p = 10
    for _ in range(18):
        m = a >= p
        if not m.any():
            break
        nd += m
        p *= 10
    return nd


def _put_int(out: np.ndarray, pos: np.ndarray, v: np.ndarray, neg: np.ndarray, nd: np.ndarray):
    """Decimal text of v at pos ('-' first where neg); returns the end positions."""
    if neg.any():
        out[pos[neg]] = ord("-")
    end = pos + neg + nd
    a = np.abs(v)
    k, p = 0, 1
    while True:
        m = nd > k
        if not m.any():
            break
        out[end[m] - 1 - k] = 48 + (a[m] // p) % 10
        k += 1
        p *= 10
    return end


def _put_lit(out: np.ndarray, pos: np.ndarray, lit: bytes):
    for k, ch in enumerate(lit):
        out[pos + k] = ch
    return pos + len(lit)


def _put_str(out: np.ndarray, pos: np.ndarray, ids: np.ndarray, tab: np.ndarray, tlen: np.ndarray):
    ln = tlen[ids]
    for k in range(tab.shape[1]):
        m = ln > k
        if not m.any():
            break
        out[pos[m] + k] = tab[ids[m], k]
    return pos + ln


def _name_table(names: List[str]):
    """(ids per entry, byte table [u, maxlen], lengths) of a name list."""
    uniq, ids = np.unique(np.asarray(names, dtype=object).astype(str), return_inverse=True)
    enc = [u.encode() for u in uniq]
    tab = np.zeros((len(enc), max(1, max((len(e) for e in enc), default=1))), np.uint8)
    for i, e in enumerate(enc):
        tab[i, :len(e)] = np.frombuffer(e, np.uint8)
    return ids.astype(np.int64), tab, np.array([len(e) for e in enc], np.int64)


def write_chains_fast(ca: ChainArrays, path: str, chunk: int = 400_000) -> None:
    """write_chains for large synthetic sets: the same bytes (chainWrite,
    kent/src/lib/chain.c:200-227), formatted with numpy a chunk of chains at
    a time.  Scores must be integer-valued (%1.0f of an integer double,
    '-0' for negative zero); otherwise this falls back to write_chains."""
    sc = np.asarray(ca.score, np.float64)
    if ca.n and not np.array_equal(sc, np.round(sc)):
        write_chains(ca, path)
        return
    tid, ttab, tlen = _name_table(ca.tname)
    qid, qtab, qlen = _name_table(ca.qname)
    with open(path, "wb") as f:
        for c0 in range(0, ca.n, chunk):
            c1 = min(ca.n, c0 + chunk)
            s = sc[c0:c1]
            sv = s.astype(np.int64)
            sneg = np.signbit(s)
            ints = {k: np.asarray(getattr(ca, k)[c0:c1], np.int64)
                    for k in ("tsize", "tstart", "tend", "qsize", "qstart", "qend", "id")}
            nd = {k: _ndig(v) for k, v in ints.items()}
            ti, qi = tid[c0:c1], qid[c0:c1]
            hlen = (6 + sneg + _ndig(sv) + 1 + tlen[ti] + 1 + nd["tsize"] + 3 + nd["tstart"] + 1
                    + nd["tend"] + 1 + qlen[qi] + 1 + nd["qsize"] + 3 + nd["qstart"] + 1
                    + nd["qend"] + 1 + nd["id"] + 1
                    + sum((v < 0).astype(np.int64) for v in ints.values()))  # '-' signs
            b0, b1 = int(ca.blk_off[c0]), int(ca.blk_off[c1])
            nb = np.diff(ca.blk_off[c0:c1 + 1])
            if (nb < 1).any():
                raise ValueError("write_chains_fast: chain without blocks")
            bt = ca.blk_t[b0:b1].astype(np.int64)
            bq = ca.blk_q[b0:b1].astype(np.int64)
            bs = ca.blk_size[b0:b1].astype(np.int64)
            last = np.zeros(b1 - b0, bool)
            last[np.cumsum(nb) - 1] = True
            dt = np.zeros(b1 - b0, np.int64)
            dq = np.zeros(b1 - b0, np.int64)
            dt[:-1] = bt[1:] - (bt[:-1] + bs[:-1])
            dq[:-1] = bq[1:] - (bq[:-1] + bs[:-1])
            dt[last] = 0
            dq[last] = 0
            ndt, ndq, nds = _ndig(dt), _ndig(dq), _ndig(bs)
            blen = np.where(last, nds + 2, nds + 3 + (dt < 0) + ndt + (dq < 0) + ndq)
            bsum = np.add.reduceat(blen, np.r_[0, np.cumsum(nb)[:-1]])
            tot = hlen + bsum
            H = np.zeros(c1 - c0, np.int64)
            np.cumsum(tot[:-1], out=H[1:])
            out = np.empty(int(tot.sum()), np.uint8)
            # headers
            p = _put_lit(out, H, b"chain ")
            p = _put_int(out, p, sv, sneg, _ndig(sv))
            p = _put_lit(out, p, b" ")
            p = _put_str(out, p, ti, ttab, tlen)
            p = _put_lit(out, p, b" ")
            p = _put_int(out, p, ints["tsize"], ints["tsize"] < 0, nd["tsize"])
            p = _put_lit(out, p, b" + ")
            p = _put_int(out, p, ints["tstart"], ints["tstart"] < 0, nd["tstart"])
            p = _put_lit(out, p, b" ")
            p = _put_int(out, p, ints["tend"], ints["tend"] < 0, nd["tend"])
            p = _put_lit(out, p, b" ")
            p = _put_str(out, p, qi, qtab, qlen)
            p = _put_lit(out, p, b" ")
            p = _put_int(out, p, ints["qsize"], ints["qsize"] < 0, nd["qsize"])
            p = _put_lit(out, p, b" ")
            out[p] = np.where(np.asarray(ca.qstrand[c0:c1]) != 0, ord("-"), ord("+"))
            p = _put_lit(out, p + 1, b" ")
            p = _put_int(out, p, ints["qstart"], ints["qstart"] < 0, nd["qstart"])
            p = _put_lit(out, p, b" ")
            p = _put_int(out, p, ints["qend"], ints["qend"] < 0, nd["qend"])
            p = _put_lit(out, p, b" ")
            p = _put_int(out, p, ints["id"], ints["id"] < 0, nd["id"])
            _put_lit(out, p, b"\n")
            # blocks
            cb = np.cumsum(blen) - blen
            ch = np.repeat(np.arange(c1 - c0), nb)
            first = np.r_[0, np.cumsum(nb)[:-1]]
            pos = H[ch] + hlen[ch] + cb - cb[first][ch]
            del cb
            e = _put_int(out, pos, bs, np.zeros(len(bs), bool), nds)
            out[e[last]] = 10
            out[e[last] + 1] = 10
            nl = ~last
            e2 = e[nl]
            out[e2] = 9
            e2 = _put_int(out, e2 + 1, dt[nl], dt[nl] < 0, ndt[nl])
            out[e2] = 9
            e2 = _put_int(out, e2 + 1, dq[nl], dq[nl] < 0, ndq[nl])
            out[e2] = 10
            f.write(out.tobytes())


def save_npz(ca: ChainArrays, path: str) -> None:
    """The arrays of a chain set (names as tables + ids), for fast reloads."""
    tid, ttab, tlen = _name_table(ca.tname)
    qid, qtab, qlen = _name_table(ca.qname)
    np.savez(path, score=ca.score, tsize=ca.tsize, tstart=ca.tstart, tend=ca.tend,
             qsize=ca.qsize, qstrand=ca.qstrand, qstart=ca.qstart, qend=ca.qend, id=ca.id,
             blk_off=ca.blk_off, blk_t=ca.blk_t, blk_q=ca.blk_q, blk_size=ca.blk_size,
             tid=tid.astype(np.int32), ttab=ttab, tlen=tlen, qid=qid.astype(np.int32), qtab=qtab,
             qlen=qlen)


def load_npz(path: str) -> ChainArrays:
    z = np.load(path)
    names = lambda tab, ln: [bytes(tab[i, :ln[i]]).decode() for i in range(len(ln))]
    tn, qn = names(z["ttab"], z["tlen"]), names(z["qtab"], z["qlen"])
    return ChainArrays(
        score=z["score"], tname=[tn[i] for i in z["tid"]], tsize=z["tsize"], tstart=z["tstart"],
        tend=z["tend"], qname=[qn[i] for i in z["qid"]], qsize=z["qsize"], qstrand=z["qstrand"],
        qstart=z["qstart"], qend=z["qend"], id=z["id"], blk_off=z["blk_off"], blk_t=z["blk_t"],
        blk_q=z["blk_q"], blk_size=z["blk_size"])
