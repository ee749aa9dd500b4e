"""Python host mirror of the reference's chain-scoring interface, on top of
the libgachain C ABI (include/gachain.h).

Reference interface                          here
-------------------------------------------  --------------------------------
gapCalcFromFile (gapCalc.c:233-255)          GapCosts(name_or_file)
axtScoreSchemeRead/Default (axt.c:423,692)   read_score_scheme(path | None)
twoBitOpen + twoBitReadSeqFrag (twoBit.c)    Engine.load_2bit(side, path)
chainRead loop (chain.c:337)                 chainfile.read_chains -> Engine.upload_chains
chainSubsetOnT + chainCalcScore (+ local)    Engine.score_ranges(chainset, ranges)
scoreChain getChainScore (scoreChain.c:207)  Engine.score_chains(chainset) (gac_score_chains)

Every scoring call runs on the GPU through libgachain; there is no CPU path.
"""
from __future__ import annotations

import ctypes as C
from typing import Iterable, Optional, Tuple

import numpy as np

from . import _lib
from ._lib import GAC_Q, GAC_T, GAC_WANT_LOCAL, ChainsetDesc, GapCalc, check, lib


def _p(a: np.ndarray) -> C.c_void_p:
    return C.c_void_p(a.ctypes.data) if a.size else C.c_void_p(0)


class GapCosts:
    """Piecewise-linear gap costs (struct gapCalc)."""

    def __init__(self, name_or_file: str = "loose"):
        self._ptr = C.POINTER(GapCalc)()
        check(lib().gac_gapcalc_build(name_or_file.encode(), C.byref(self._ptr)))
        self.name = name_or_file

    @property
    def ptr(self):
        return self._ptr

    def cost(self, dq: int, dt: int) -> int:
        """gapCalcCost on the host (gac_gap_cost)."""
        return int(lib().gac_gap_cost(self._ptr, int(dq), int(dt)))

    def tables(self):
        g = self._ptr.contents
        n, m = g.small_size, g.long_count
        return {
            "small_size": n,
            "q_small": np.ctypeslib.as_array(g.q_small, (n,)).copy(),
            "t_small": np.ctypeslib.as_array(g.t_small, (n,)).copy(),
            "b_small": np.ctypeslib.as_array(g.b_small, (n,)).copy(),
            "long_pos": np.ctypeslib.as_array(g.long_pos, (m,)).copy(),
        }

    def __del__(self):
        try:
            if self._ptr:
                lib().gac_gapcalc_free(self._ptr)
        except Exception:
            pass


def read_score_scheme(path: Optional[str] = None) -> Tuple[np.ndarray, int, int, str]:
    """Returns (mat[4,4] int32 [query][target] in A,C,G,T order, gapOpen,
    gapExtend, extra)."""
    mat = (C.c_int32 * 16)()
    go, ge = C.c_int32(), C.c_int32()
    extra = C.c_void_p()
    check(lib().gac_scheme_read(path.encode() if path else None, mat, C.byref(go),
                                C.byref(ge), C.byref(extra)))
    ex = ""
    if extra.value:
        ex = C.string_at(extra.value).decode()
        C.CDLL(None).free(extra)
    return np.array(mat[:], dtype=np.int32).reshape(4, 4), go.value, ge.value, ex


class ChainSet:
    def __init__(self, engine: "Engine", handle: C.c_void_p, n_chains: int, n_blocks: int,
                 aligned_bases: int):
        self.engine = engine
        self.handle = handle
        self.n_chains = n_chains
        self.n_blocks = n_blocks
        self.aligned_bases = aligned_bases

    def close(self):
        if self.handle:
            lib().gac_chains_free(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Engine:
    """One libgachain context on one MI355X (gfx950) device."""

    def __init__(self, device: int = 0):
        h = C.c_void_p()
        check(lib().gac_open(device, C.byref(h)))
        self.h = h
        self.device = device

    @property
    def arch(self) -> str:
        return lib().gac_device_arch(self.h).decode()

    def close(self):
        if self.h:
            lib().gac_close(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- scoring scheme
    def set_scoring(self, mat: np.ndarray, gap: GapCosts) -> None:
        m = np.ascontiguousarray(np.asarray(mat, dtype=np.int32).reshape(16))
        check(lib().gac_set_scoring(self.h, m.ctypes.data_as(C.POINTER(C.c_int32)), gap.ptr))
        self._gap = gap

    # ---- genomes
    def load_2bit(self, side: int, path: str) -> None:
        check(lib().gac_genome_load_2bit(self.h, side, path.encode()))

    def add_sequences(self, side: int, seqs: Iterable) -> None:
        """seqs: iterable of (name, size, packed uint8 .2bit payload, n_starts, n_sizes)."""
        for name, size, packed, ns, nz in seqs:
            packed = np.ascontiguousarray(packed, dtype=np.uint8)
            ns = np.ascontiguousarray(ns, dtype=np.int32)
            nz = np.ascontiguousarray(nz, dtype=np.int32)
            check(lib().gac_genome_add_seq(self.h, side, name.encode(), int(size), _p(packed),
                                           len(ns), _p(ns), _p(nz)))
        check(lib().gac_genome_finalize(self.h, side))

    def seq_index(self, side: int, name: str) -> int:
        return lib().gac_genome_seq_index(self.h, side, name.encode())

    def seq_size(self, side: int, idx: int) -> int:
        return lib().gac_genome_seq_size(self.h, side, idx)

    def seq_count(self, side: int) -> int:
        return lib().gac_genome_seq_count(self.h, side)

    def decode(self, side: int, idx: int, start: int, end: int) -> str:
        buf = C.create_string_buffer(max(end - start, 1))
        check(lib().gac_genome_decode(self.h, side, idx, start, end, buf))
        return buf.raw[: end - start].decode()

    # ---- chains
    def upload_chains(self, ca) -> ChainSet:
        """Upload a chainfile.ChainArrays; sequences are resolved by name."""
        tidx = np.array([self.seq_index(GAC_T, n) for n in ca.tname], dtype=np.int32)
        qidx = np.array([self.seq_index(GAC_Q, n) for n in ca.qname], dtype=np.int32)
        if (tidx < 0).any() or (qidx < 0).any():
            bad = [n for n, i in zip(ca.tname, tidx) if i < 0] + \
                  [n for n, i in zip(ca.qname, qidx) if i < 0]
            raise KeyError(f"sequence(s) not loaded: {sorted(set(bad))[:5]}")
        return self.upload_chain_arrays(tidx, qidx, ca.qstrand, ca.blk_off, ca.blk_t, ca.blk_q,
                                        ca.blk_size)

    @staticmethod
    def _desc(t_seq, q_seq, q_strand, blk_off, blk_t, blk_q, blk_size):
        """(gac_chainset_desc, the arrays it points into: keep them alive)"""
        arrs = [np.ascontiguousarray(t_seq, np.int32), np.ascontiguousarray(q_seq, np.int32),
                np.ascontiguousarray(q_strand, np.uint8), np.ascontiguousarray(blk_off, np.int64),
                np.ascontiguousarray(blk_t, np.int32), np.ascontiguousarray(blk_q, np.int32),
                np.ascontiguousarray(blk_size, np.int32)]
        d = ChainsetDesc()
        d.n_chains = len(arrs[0])
        d.t_seq, d.q_seq, d.q_strand, d.blk_off = (_p(a) for a in arrs[:4])
        d.n_blocks = len(arrs[4])
        d.blk_t, d.blk_q, d.blk_size = (_p(a) for a in arrs[4:])
        return d, arrs

    def upload_chain_arrays(self, t_seq, q_seq, q_strand, blk_off, blk_t, blk_q, blk_size) -> ChainSet:
        d, arrs = self._desc(t_seq, q_seq, q_strand, blk_off, blk_t, blk_q, blk_size)
        h = C.c_void_p()
        check(lib().gac_chains_upload(self.h, C.byref(d), C.byref(h)))
        return ChainSet(self, h, d.n_chains, d.n_blocks, int(arrs[6].sum(dtype=np.int64)))

    def reupload_chain_arrays(self, cs: ChainSet, t_seq, q_seq, q_strand, blk_off, blk_t, blk_q,
                              blk_size) -> ChainSet:
        """gac_chains_reupload: cs now holds these chains (its memory reused)."""
        d, arrs = self._desc(t_seq, q_seq, q_strand, blk_off, blk_t, blk_q, blk_size)
        check(lib().gac_chains_reupload(self.h, C.byref(d), cs.handle))
        cs.n_chains, cs.n_blocks = d.n_chains, d.n_blocks
        cs.aligned_bases = int(arrs[6].sum(dtype=np.int64))
        return cs

    def score_ranges_host(self, t_seq, q_seq, q_strand, blk_off, blk_t, blk_q, blk_size,
                          ranges: np.ndarray, want_local: bool = False):
        """gac_score_ranges_host: ranges of chains held in host memory."""
        d, arrs = self._desc(t_seq, q_seq, q_strand, blk_off, blk_t, blk_q, blk_size)
        r = np.ascontiguousarray(np.asarray(ranges, dtype=np.int32).reshape(-1, 3))
        n = r.shape[0]
        g = np.zeros(n, np.int64)
        ali = np.zeros(n, np.int32)
        loc = np.zeros(n, np.int64) if want_local else None
        check(lib().gac_score_ranges_host(self.h, C.byref(d), _p(r), n,
                                          GAC_WANT_LOCAL if want_local else 0, _p(g),
                                          _p(loc) if want_local else None, _p(ali)))
        return g, loc, ali

    # ---- scoring
    def score_ranges(self, cs: ChainSet, ranges: np.ndarray, want_local: bool = False):
        """ranges: int32 [n, 3] (chain, tStart, tEnd).  Returns (global int64,
        local int64 or None, ali int32)."""
        r = np.ascontiguousarray(np.asarray(ranges, dtype=np.int32).reshape(-1, 3))
        n = r.shape[0]
        g = np.zeros(n, np.int64)
        ali = np.zeros(n, np.int32)
        loc = np.zeros(n, np.int64) if want_local else None
        check(lib().gac_score_ranges(self.h, cs.handle, _p(r), n,
                                     GAC_WANT_LOCAL if want_local else 0, _p(g),
                                     _p(loc) if want_local else None, _p(ali)))
        return g, loc, ali

    def score_windows(self, cs: ChainSet, windows: np.ndarray, want_local: bool = False):
        """windows: int32 [n, 5] (chain, tStart, tEnd, first block, block count;
        gac_window).  Returns as score_ranges."""
        w = np.ascontiguousarray(np.asarray(windows, dtype=np.int32).reshape(-1, 5))
        n = w.shape[0]
        g = np.zeros(n, np.int64)
        ali = np.zeros(n, np.int32)
        loc = np.zeros(n, np.int64) if want_local else None
        check(lib().gac_score_windows(self.h, cs.handle, _p(w), n,
                                      GAC_WANT_LOCAL if want_local else 0, _p(g),
                                      _p(loc) if want_local else None, _p(ali)))
        return g, loc, ali

    def full_ranges(self, ca) -> np.ndarray:
        return np.stack([np.arange(ca.n, dtype=np.int32), ca.tstart.astype(np.int32),
                         ca.tend.astype(np.int32)], axis=1)

    def score_chains(self, cs: ChainSet, ca=None, want_local: bool = True):
        """scoreChain: global, local and aligned bases of every chain of the
        set, in order (gac_score_chains: the set's own plan, no ranges)."""
        n = cs.n_chains
        g = np.zeros(n, np.int64)
        ali = np.zeros(n, np.int32)
        loc = np.zeros(n, np.int64) if want_local else None
        check(lib().gac_score_chains(self.h, cs.handle, GAC_WANT_LOCAL if want_local else 0,
                                     _p(g), _p(loc) if want_local else None, _p(ali)))
        return g, loc, ali

    def score_chains_device(self, cs: ChainSet, d_g: int, d_ali: int, d_l: int = 0,
                            want_local: bool = False, stream: int = 0) -> None:
        check(lib().gac_score_chains_device(
            self.h, cs.handle, GAC_WANT_LOCAL if want_local else 0, C.c_void_p(d_g),
            C.c_void_p(d_l) if d_l else None, C.c_void_p(d_ali),
            C.c_void_p(stream) if stream else None))

    # ---- device buffers / timing (bench)
    def dev_alloc(self, nbytes: int) -> int:
        p = C.c_void_p()
        check(lib().gac_dev_alloc(self.h, nbytes, C.byref(p)))
        return p.value

    def dev_free(self, p: int) -> None:
        check(lib().gac_dev_free(self.h, C.c_void_p(p)))

    def h2d(self, dst: int, a: np.ndarray) -> None:
        a = np.ascontiguousarray(a)
        check(lib().gac_memcpy_h2d(self.h, C.c_void_p(dst), _p(a), a.nbytes))

    def d2h(self, a: np.ndarray, src: int) -> None:
        check(lib().gac_memcpy_d2h(self.h, _p(a), C.c_void_p(src), a.nbytes))

    def score_ranges_device(self, cs: ChainSet, d_ranges: int, n: int, d_g: int, d_ali: int,
                            d_l: int = 0, want_local: bool = False, stream: int = 0) -> None:
        check(lib().gac_score_ranges_device(
            self.h, cs.handle, C.c_void_p(d_ranges), n, GAC_WANT_LOCAL if want_local else 0,
            C.c_void_p(d_g), C.c_void_p(d_l) if d_l else None, C.c_void_p(d_ali),
            C.c_void_p(stream) if stream else None))

    def score_windows_device(self, cs: ChainSet, d_windows: int, n: int, d_g: int, d_ali: int,
                             d_l: int = 0, want_local: bool = False, stream: int = 0) -> None:
        check(lib().gac_score_windows_device(
            self.h, cs.handle, C.c_void_p(d_windows), n, GAC_WANT_LOCAL if want_local else 0,
            C.c_void_p(d_g), C.c_void_p(d_l) if d_l else None, C.c_void_p(d_ali),
            C.c_void_p(stream) if stream else None))

    def synchronize(self) -> None:
        check(lib().gac_synchronize(self.h))

    def prof_enable(self, on: bool = True, kernels=None) -> None:
        """Time launches with HIP events: all kernels, or those in `kernels`
        (GAC_K_* ids)."""
        mask = 0
        if on:
            mask = (1 << 3) - 1 if kernels is None else sum(1 << k for k in kernels)
        check(lib().gac_prof_enable(self.h, mask))

    def prof_reset(self) -> None:
        check(lib().gac_prof_reset(self.h))

    def prof_read(self, k: int):
        ms, n = C.c_double(), C.c_int64()
        check(lib().gac_prof_read(self.h, k, C.byref(ms), C.byref(n)))
        return ms.value, n.value


__all__ = ["Engine", "ChainSet", "GapCosts", "read_score_scheme", "GAC_T", "GAC_Q"]
