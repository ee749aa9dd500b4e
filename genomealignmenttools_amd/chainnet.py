"""chainNet (with -rescore) on the libgachain netting engine + GPU scorer.

Python mirror of src/chainNet/chainNet.c's chainNet() flow (:918-1002):
net the score-sorted chains on the host (gac_net_build), rescore the partial
target-side fills on the GPU (gac_score_ranges), write both nets
(gac_net_write).  The C tool bin/chainNet does the same from the command line.
"""
from __future__ import annotations

import ctypes as C
from typing import Dict, List, Optional

import numpy as np

from ._lib import GAC_Q, GAC_T, NetInput, NetOpts, check, lib


def _p(a):
    return C.c_void_p(a.ctypes.data) if a.size else C.c_void_p(0)


class Net:
    """A built net (both sides).  Keeps the borrowed input arrays alive."""

    def __init__(self, ca, tsizes: Dict[str, int], qsizes: Dict[str, int], min_score: float,
                 min_space: int = 25, min_fill: Optional[int] = None, incl_hap: bool = False,
                 sides: int = (1 << GAC_T) | (1 << GAC_Q)):
        tnames = list(tsizes)
        qnames = list(qsizes)
        tix = {n: i for i, n in enumerate(tnames)}
        qix = {n: i for i, n in enumerate(qnames)}
        self._keep = []

        def keep(a, dt):
            a = np.ascontiguousarray(a, dt)
            self._keep.append(a)
            return a
        n = ca.n
        self.tnames_c = (C.c_char_p * max(1, len(tnames)))(*[x.encode() for x in tnames])
        self.qnames_c = (C.c_char_p * max(1, len(qnames)))(*[x.encode() for x in qnames])
        inp = NetInput()
        inp.n_chains = n
        inp.score = _p(keep(ca.score, np.float64))
        inp.id = _p(keep(ca.id, np.int32))
        inp.t_seq = _p(keep([tix[x] for x in ca.tname], np.int32))
        inp.q_seq = _p(keep([qix[x] for x in ca.qname], np.int32))
        inp.q_strand = _p(keep(ca.qstrand, np.uint8))
        inp.t_start = _p(keep(ca.tstart, np.int32))
        inp.t_end = _p(keep(ca.tend, np.int32))
        inp.q_start = _p(keep(ca.qstart, np.int32))
        inp.q_end = _p(keep(ca.qend, np.int32))
        inp.blk_off = _p(keep(ca.blk_off, np.int64))
        inp.blk_t = _p(keep(ca.blk_t, np.int32))
        inp.blk_q = _p(keep(ca.blk_q, np.int32))
        inp.blk_size = _p(keep(ca.blk_size, np.int32))
        inp.n_tseq = len(tnames)
        inp.t_names = C.cast(self.tnames_c, C.c_void_p)
        inp.t_sizes = _p(keep([tsizes[x] for x in tnames], np.int32))
        inp.n_qseq = len(qnames)
        inp.q_names = C.cast(self.qnames_c, C.c_void_p)
        inp.q_sizes = _p(keep([qsizes[x] for x in qnames], np.int32))
        self._inp = inp
        opt = NetOpts(min_space, min_space // 2 if min_fill is None else min_fill,
                      float(min_score), 1 if incl_hap else 0)
        self.opts = opt
        h = C.c_void_p()
        check(lib().gac_net_build_sides(C.byref(inp), C.byref(opt), sides, C.byref(h)))
        self.h = h

    @property
    def netted(self) -> int:
        return lib().gac_net_netted(self.h)

    def fills(self, side: int = GAC_T):
        n = lib().gac_net_fill_count(self.h, side)
        out = {k: np.zeros(n, np.int32) for k in ("chain", "start", "end", "ali")}
        flags = np.zeros(n, np.uint8)
        check(lib().gac_net_get_fills(self.h, side, _p(out["chain"]), _p(out["start"]),
                                      _p(out["end"]), _p(out["ali"]), _p(flags)))
        out["flags"] = flags
        if side == GAC_T:  # chainSubsetOnT's window of every target fill
            out["first_block"] = np.zeros(n, np.int32)
            out["n_blocks"] = np.zeros(n, np.int32)
            check(lib().gac_net_get_fill_windows(self.h, side, _p(out["first_block"]),
                                                 _p(out["n_blocks"])))
        return out

    def rescore_windows(self):
        """gac_net_rescore_windows: the partial, printed target fills in
        pre-order as gac_window records [n, 5] (chain, start, end, first
        block, block count) and their pre-order positions."""
        w = C.c_void_p()
        pos = C.c_void_p()
        n = C.c_int64()
        check(lib().gac_net_rescore_windows(self.h, GAC_T, C.byref(w), C.byref(pos), C.byref(n)))
        m = n.value
        try:
            win = np.ctypeslib.as_array(C.cast(w, C.POINTER(C.c_int32)), (max(m, 1) * 5,))
            ps = np.ctypeslib.as_array(C.cast(pos, C.POINTER(C.c_int64)), (max(m, 1),))
            return win[:m * 5].reshape(m, 5).copy(), ps[:m].copy()
        finally:
            libc = C.CDLL(None)
            libc.free(w)
            libc.free(pos)

    def write(self, side: int, path: str, t_scores: Optional[np.ndarray] = None,
              meta: Optional[List[str]] = None) -> None:
        meta = meta or []
        marr = (C.c_char_p * max(1, len(meta)))(*[m.encode() for m in meta])
        ts = None
        if t_scores is not None:
            ts = np.ascontiguousarray(t_scores, np.int64)
            self._keep.append(ts)
        check(lib().gac_net_write(self.h, side, _p(ts) if ts is not None else None,
                                  path.encode(), C.cast(marr, C.c_void_p), len(meta)))

    def close(self):
        if getattr(self, "h", None):
            lib().gac_net_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def net_fills(ca, tsizes, qsizes, min_score: float = 0.0, **kw):
    """Net the chains and return the rescore work list of the T side:
    dict(chain, start, end, ali, partial (bool), visible (bool),
    netted_chains).  With -rescore the GPU scores fills that are partial and
    visible (exactly those whose score chainNet prints)."""
    net = Net(ca, tsizes, qsizes, min_score, **kw)
    f = net.fills(GAC_T)
    f["partial"] = ((f["flags"] & 1) != 0) & ((f["flags"] & 2) != 0)
    f["netted_chains"] = net.netted
    f["net"] = net
    return f


def chain_net_rescore(engine, cs, ca, tsizes, qsizes, t_net: str, q_net: str,
                      rescore: bool = True, min_score: Optional[float] = None, **kw):
    """Full chainNet [-rescore]: returns the Net."""
    ms = 0.0 if rescore else (2000.0 if min_score is None else min_score)
    net = Net(ca, tsizes, qsizes, ms, **kw)
    scores = None
    if rescore:
        f = net.fills(GAC_T)
        sel = np.nonzero(((f["flags"] & 1) != 0) & ((f["flags"] & 2) != 0))[0]
        scores = np.zeros(len(f["chain"]), np.int64)
        if len(sel):
            R = np.stack([f["chain"][sel], f["start"][sel], f["end"][sel]], 1)
            g, _, _ = engine.score_ranges(cs, R)
            scores[sel] = g
    net.write(GAC_T, t_net, scores, ca.meta)
    net.write(GAC_Q, q_net, None, ca.meta)
    return net
