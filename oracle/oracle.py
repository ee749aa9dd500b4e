"""CPU ORACLE wrappers -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
import this module, and only as the checker / baseline, never as the thing
measured or shipped.

  * libgacoracle.so  (oracle/gac_oracle.c): plain-C restatement of the
    reference scoring path; pinned by tests/test_oracle.py against the
    reference itself.
  * libkentref.so    (oracle/_ref, built from /root/reference by oracle/ref.mk):
    the reference's own kent objects driven by oracle/ref_harness.c.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from typing import Dict, Optional

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
ORACLE_SO = os.path.join(HERE, "_build", "libgacoracle.so")
REF_DIR = os.path.join(HERE, "_ref")
KENTREF_SO = os.path.join(REF_DIR, "libkentref.so")

_olib = None
_klib = None


def _p(a):
    return C.c_void_p(a.ctypes.data) if a.size else C.c_void_p(0)


def olib():
    global _olib
    if _olib is None:
        if not os.path.exists(ORACLE_SO):
            subprocess.run(["make", "-C", REPO, "oracle"], check=True, capture_output=True)
        L = C.CDLL(ORACLE_SO)
        L.or_gap_new.restype = C.c_void_p
        L.or_gap_new.argtypes = [C.c_char_p]
        L.or_gap_cost.restype = C.c_int
        L.or_gap_cost.argtypes = [C.c_void_p, C.c_int, C.c_int]
        L.or_gap_costs.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p]
        L.or_matrix_new.restype = C.c_void_p
        L.or_matrix_new.argtypes = [C.c_void_p]
        L.or_free.argtypes = [C.c_void_p]
        L.or_subchain.restype = C.c_int
        L.or_subchain.argtypes = [C.c_char_p, C.c_char_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                  C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_void_p,
                                  C.POINTER(C.c_longlong), C.POINTER(C.c_longlong),
                                  C.POINTER(C.c_int)]
        L.or_twobit_load.restype = C.c_void_p
        L.or_twobit_load.argtypes = [C.c_char_p]
        L.or_twobit_count.restype = C.c_int
        L.or_twobit_count.argtypes = [C.c_void_p]
        L.or_twobit_name.restype = C.c_char_p
        L.or_twobit_name.argtypes = [C.c_void_p, C.c_int]
        L.or_twobit_size.restype = C.c_int
        L.or_twobit_size.argtypes = [C.c_void_p, C.c_int]
        L.or_twobit_seq.restype = C.c_void_p
        L.or_twobit_seq.argtypes = [C.c_void_p, C.c_int]
        L.or_revcomp.argtypes = [C.c_char_p, C.c_int, C.c_char_p]
        _olib = L
    return _olib


class OracleGap:
    def __init__(self, name: str):
        self.h = olib().or_gap_new(name.encode())
        if not self.h:
            raise ValueError(f"oracle can't read gap costs {name}")

    def cost(self, dq: int, dt: int) -> int:
        return olib().or_gap_cost(self.h, int(dq), int(dt))

    def costs(self, dq: np.ndarray, dt: np.ndarray) -> np.ndarray:
        dq = np.ascontiguousarray(dq, np.int32)
        dt = np.ascontiguousarray(dt, np.int32)
        out = np.zeros(len(dq), np.int32)
        olib().or_gap_costs(self.h, len(dq), _p(dq), _p(dt), _p(out))
        return out


def read_2bit_text(path: str) -> Dict[str, bytes]:
    """Whole-sequence decode of a .2bit file ('acgtn' bytes per name)."""
    L = olib()
    h = L.or_twobit_load(path.encode())
    if not h:
        raise ValueError(f"oracle can't read {path}")
    out = {}
    for i in range(L.or_twobit_count(h)):
        n = L.or_twobit_size(h, i)
        out[L.or_twobit_name(h, i).decode()] = C.string_at(L.or_twobit_seq(h, i), n)
    return out


def revcomp(s: bytes) -> bytes:
    out = C.create_string_buffer(len(s))
    olib().or_revcomp(s, len(s), out)
    return out.raw


class OracleScorer:
    """chainSubsetOnT + chainCalcScore + chainCalcScoreLocal on 1-byte text."""

    def __init__(self, tseqs: Dict[str, bytes], qseqs: Dict[str, bytes], mat16, gap: str):
        self.t = tseqs
        self.q = qseqs
        self.qrc: Dict[str, bytes] = {}
        m = np.ascontiguousarray(np.asarray(mat16, np.int32).reshape(16))
        self.m = olib().or_matrix_new(_p(m))
        self._m_keep = m
        self.gap = OracleGap(gap)

    def qseq(self, name: str, minus: bool) -> bytes:
        if not minus:
            return self.q[name]
        if name not in self.qrc:
            self.qrc[name] = revcomp(self.q[name])
        return self.qrc[name]

    def score_ranges(self, ca, ranges):
        ranges = np.asarray(ranges, np.int64).reshape(-1, 3)
        n = len(ranges)
        g = np.zeros(n, np.int64)
        l = np.zeros(n, np.int64)
        a = np.zeros(n, np.int32)
        gg, ll, aa = C.c_longlong(), C.c_longlong(), C.c_int()
        L = olib()
        for i, (c, s, e) in enumerate(ranges):
            bt, bq, bs = (np.ascontiguousarray(x, np.int32) for x in ca.blocks(int(c)))
            L.or_subchain(self.t[ca.tname[c]], self.qseq(ca.qname[c], bool(ca.qstrand[c])),
                          _p(bt), _p(bq), _p(bs), len(bs), int(s), int(e), self.m,
                          self.gap.h, C.byref(gg), C.byref(ll), C.byref(aa))
            g[i], l[i], a[i] = gg.value, ll.value, aa.value
        return g, l, a


def genome_text(gen) -> Dict[str, bytes]:
    """synth.Genome -> {name: 'acgtn' bytes}."""
    return {n: gen.text(i).encode() for i, n in enumerate(gen.names)}


# ------------------------------------------------------------- reference
KENTREF = os.path.join(REF_DIR, "kentref")


def have_ref() -> bool:
    return os.path.exists(KENTREF)


def ref_tool(name: str) -> str:
    return os.path.join(REF_DIR, name)


def _run_kentref(args, timeout=3600):
    import json
    out = subprocess.run([KENTREF] + args, capture_output=True, text=True, timeout=timeout)
    if out.returncode != 0:
        raise RuntimeError(f"kentref {args[0]} failed: {out.stderr[-2000:]}")
    return json.loads(out.stdout.strip().splitlines()[-1])


class KentRef:
    """The reference's own kent code (oracle/_ref/kentref) on a chain file +
    two .2bit files."""

    def __init__(self, chain_file: str, t2bit: str, q2bit: str, scheme: Optional[str],
                 gap: str):
        self.args = [chain_file, t2bit, q2bit, scheme or "-", gap]
        self.last_seconds = None

    def _run(self, mode, ranges, tmpdir=None):
        import tempfile
        r = np.ascontiguousarray(np.asarray(ranges, np.int32).reshape(-1, 3))
        with tempfile.TemporaryDirectory(dir=tmpdir) as d:
            rin, rout = os.path.join(d, "r.bin"), os.path.join(d, "o.bin")
            r.tofile(rin)
            info = _run_kentref([mode] + self.args + [rin, rout])
            self.last_seconds = info["seconds"]
            raw = open(rout, "rb").read()
        return raw, len(r)

    def rescore_fills(self, ranges):
        raw, n = self._run("rescore", ranges)
        sc = np.frombuffer(raw[: 8 * n], np.float64).copy()
        ali = np.frombuffer(raw[8 * n:], np.int32).copy()
        return sc, ali

    def subchain_scores(self, ranges):
        raw, n = self._run("subchain", ranges)
        g = np.frombuffer(raw[: 8 * n], np.float64).copy()
        l = np.frombuffer(raw[8 * n: 16 * n], np.float64).copy()
        ali = np.frombuffer(raw[16 * n:], np.int32).copy()
        return g, l, ali


def kent_gap_costs(gap: str, dq, dt) -> np.ndarray:
    import tempfile
    pairs = np.ascontiguousarray(np.stack([np.asarray(dq, np.int32), np.asarray(dt, np.int32)], 1))
    with tempfile.TemporaryDirectory() as d:
        pin, pout = os.path.join(d, "p.bin"), os.path.join(d, "o.bin")
        pairs.tofile(pin)
        _run_kentref(["gapcost", gap, pin, pout])
        return np.fromfile(pout, np.int32)
