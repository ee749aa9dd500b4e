#!/usr/bin/env python3
"""Probe (analysis only, no GPU): HBM line traffic of k_tile on the C5 fills
under alternative layouts and orders, by replaying the kernel's accesses
through a per-XCD set-associative LRU model of the 4 MiB L2s.

Inputs: a C5 directory from gac_synth (chains.bin, *.sizes) and the fills
the tool rescored (GAC_DUMP_RANGES=fills.bin; the CPU stand-in
oracle/_build/chainNet_cpu dumps the same list).  Model of the launch: flat
window blocks in submission order, 64 per tile; tile t runs on XCD
(t mod 6144) // 768 in wave step t // 6144 (the persistent grid of 1536
workgroups x 4 waves and k_tile's XCD-aware tile mapping); per block the
RangeDesc line (first block of a range), the block record line, and the
target / query plane lines its 32-base chunks read (16-B loads: words w,
w + 1).  Misses of the model = lines read from beyond L2 (what
TCC_EA0_RDREQ counts).

usage: sim.py C5DIR [--order net|chain|chaint] [--brec 16|12|8] [--rdesc 32|16]
"""
import argparse
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))


def sizes(p):
    sz = []
    for line in open(p):
        sz.append(int(line.split()[1]))
    return np.array(sz, np.int64)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("c5")
    ap.add_argument("--order", default="net")
    ap.add_argument("--brec", type=int, default=16)
    ap.add_argument("--rdesc", type=int, default=32)
    a = ap.parse_args()
    from bench import load_chains_bin
    ch = load_chains_bin(a.c5)
    n = ch["n"]
    f = np.fromfile(os.path.join(a.c5, "fills.bin"), np.int32).reshape(-1, 3).astype(np.int64)
    fc, fs, fe = f[:, 0], f[:, 1], f[:, 2]
    ts, qs = sizes(os.path.join(a.c5, "t.sizes")), sizes(os.path.join(a.c5, "q.sizes"))
    twoff = np.concatenate([[0], np.cumsum((ts + 31) // 32)])
    qwoff = np.concatenate([[0], np.cumsum((qs + 31) // 32)])
    off = ch["off"]
    bt, bq, bs = (ch[k].astype(np.int64) for k in ("bt", "bq", "bs"))
    cid = np.repeat(np.arange(n, dtype=np.int64), np.diff(off))
    first = np.searchsorted((cid << 32) | (bt + bs), (fc << 32) | fs, "right")
    last = np.searchsorted((cid << 32) | bt, (fc << 32) | fe, "left") - 1
    nw = np.maximum(last - first + 1, 0)
    del cid
    nf = len(fc)
    if a.order == "net":
        perm = np.arange(nf)
    elif a.order == "chain":
        perm = np.lexsort((np.arange(nf), fc))
    elif a.order == "chaint":
        perm = np.lexsort((np.arange(nf), fc, ch["tstart"][fc], ch["tseq"][fc]))
    else:
        raise SystemExit(a.order)
    nwp = nw[perm]
    nb = int(nwp.sum())
    fpos = np.repeat(np.arange(nf), nwp)
    kin = np.arange(nb) - np.repeat(np.cumsum(nwp) - nwp, nwp)
    c = fc[perm][fpos]
    gbi = first[perm][fpos] + kin  # (global block index: first is global)
    s, e = fs[perm][fpos], fe[perm][fpos]
    t0, q0, z = bt[gbi], bq[gbi], bs[gbi]
    cts = np.maximum(t0, s)
    cqs = q0 + (cts - t0)
    ln = np.minimum(t0 + z, e) - cts
    minus = ch["strand"][c].astype(bool)
    tg = twoff[ch["tseq"][c]] * 32 + cts
    qsz = qs[ch["qseq"][c]]
    qg = qwoff[ch["qseq"][c]] * 32 + np.where(minus, qsz - cqs - ln, cqs)
    del cts, cqs, t0, q0, z, s, e, minus, qsz

    def lines(p, l):
        return (p // 32) // 16, ((p + np.maximum(l, 1) - 1) // 32 + 1) // 16
    tl0, tl1 = lines(tg, ln)
    ql0, ql1 = lines(qg, ln)
    del tg, qg, ln
    tile = np.arange(nb) // 64
    xcd = (tile % 6144) // 768
    key = (xcd << 40) | (tile // 6144)
    firstblk = np.r_[True, fpos[1:] != fpos[:-1]]
    nt, nq = tl1 - tl0 + 1, ql1 - ql0 + 1
    cnt = 1 + firstblk + nt + nq
    tot = int(cnt.sum())
    owner = np.repeat(np.arange(nb), cnt)
    k = np.arange(tot) - np.repeat(np.cumsum(cnt) - cnt, cnt)
    k -= firstblk[owner]  # -1: the RangeDesc, 0: block record, then target, query lines
    out = np.empty(tot, np.uint64)
    m = k == -1
    out[m] = (fpos[owner[m]] * a.rdesc // 128 + (3 << 40)).astype(np.uint64)
    m = k == 0
    out[m] = (gbi[owner[m]] * a.brec // 128 + (2 << 40)).astype(np.uint64)
    m = (k >= 1) & (k <= nt[owner])
    out[m] = (tl0[owner[m]] + k[m] - 1).astype(np.uint64)
    m = k > nt[owner]
    out[m] = (ql0[owner[m]] + k[m] - 1 - nt[owner[m]] + (1 << 40)).astype(np.uint64)
    o = np.argsort(key[owner], kind="stable")
    rec = np.empty((tot, 2), np.uint64)
    rec[:, 0] = (key[owner][o] >> 40).astype(np.uint64)
    rec[:, 1] = out[o]
    exe = os.path.join(tempfile.gettempdir(), "gac_lru_sim")
    subprocess.run(["gcc", "-O2", "-o", exe, os.path.join(HERE, "lru.c")], check=True)
    with tempfile.NamedTemporaryFile(suffix=".bin") as tf:
        rec.tofile(tf.name)
        del rec, out
        r = subprocess.run([exe, tf.name], capture_output=True, text=True, check=True)
    names = {"region 0": "target planes", "region 1": "query planes", "region 2": "block records",
             "region 3": "RangeDesc"}
    txt = r.stdout
    for kk, v in names.items():
        txt = txt.replace(kk + ":", v + ":")
    print(f"order={a.order} brec={a.brec} rdesc={a.rdesc}: {nf} fills, {nb} window blocks")
    print(txt, end="")


if __name__ == "__main__":
    main()
