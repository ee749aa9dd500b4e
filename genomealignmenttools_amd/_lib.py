"""ctypes binding of libgachain (include/gachain.h).

The library is built in-tree by ``make`` (``genomealignmenttools_amd/lib/
libgachain.so``).  Loading fails loudly when it is missing or unbuildable:
there is no Python or CPU fallback for any scoring entry point.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
import threading

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
REPO_DIR = os.path.dirname(PKG_DIR)
LIB_DIR = os.path.join(PKG_DIR, "lib")
LIB_PATH = os.path.join(LIB_DIR, "libgachain.so")
# A/B probes only: GAC_LIB_VARIANT=NAME loads lib/variants/NAME/libgachain.so
# (built by `make variant NAME=... VFLAGS=...`; the tools keep lib/).
if os.environ.get("GAC_LIB_VARIANT"):
    LIB_PATH = os.path.join(LIB_DIR, "variants", os.environ["GAC_LIB_VARIANT"], "libgachain.so")
BIN_DIR = os.path.join(PKG_DIR, "bin")

GAC_OK = 0
GAC_T = 0
GAC_Q = 1
GAC_WANT_LOCAL = 1
GAC_K_PLAN, GAC_K_TILE, GAC_K_COMBINE = 0, 1, 2

_lock = threading.Lock()
_lib = None


class GacError(RuntimeError):
    """Error returned by libgachain (message from gac_last_error())."""

    def __init__(self, code: int, msg: str):
        super().__init__(f"libgachain error {code}: {msg}")
        self.code = code


class GapCalc(C.Structure):
    _fields_ = [
        ("small_size", C.c_int32),
        ("long_count", C.c_int32),
        ("q_small", C.POINTER(C.c_int32)),
        ("t_small", C.POINTER(C.c_int32)),
        ("b_small", C.POINTER(C.c_int32)),
        ("long_pos", C.POINTER(C.c_int32)),
        ("q_long", C.POINTER(C.c_double)),
        ("t_long", C.POINTER(C.c_double)),
        ("b_long", C.POINTER(C.c_double)),
        ("q_last_pos", C.c_int32),
        ("t_last_pos", C.c_int32),
        ("b_last_pos", C.c_int32),
        ("q_last_val", C.c_double),
        ("t_last_val", C.c_double),
        ("b_last_val", C.c_double),
        ("q_last_slope", C.c_double),
        ("t_last_slope", C.c_double),
        ("b_last_slope", C.c_double),
    ]


class ChainsetDesc(C.Structure):
    _fields_ = [
        ("n_chains", C.c_int64),
        ("t_seq", C.c_void_p),
        ("q_seq", C.c_void_p),
        ("q_strand", C.c_void_p),
        ("blk_off", C.c_void_p),
        ("n_blocks", C.c_int64),
        ("blk_t", C.c_void_p),
        ("blk_q", C.c_void_p),
        ("blk_size", C.c_void_p),
    ]


class NetInput(C.Structure):
    _fields_ = [
        ("n_chains", C.c_int64),
        ("score", C.c_void_p), ("id", C.c_void_p), ("t_seq", C.c_void_p),
        ("q_seq", C.c_void_p), ("q_strand", C.c_void_p),
        ("t_start", C.c_void_p), ("t_end", C.c_void_p), ("q_start", C.c_void_p),
        ("q_end", C.c_void_p), ("blk_off", C.c_void_p), ("blk_t", C.c_void_p),
        ("blk_q", C.c_void_p), ("blk_size", C.c_void_p),
        ("n_tseq", C.c_int32), ("t_names", C.c_void_p), ("t_sizes", C.c_void_p),
        ("n_qseq", C.c_int32), ("q_names", C.c_void_p), ("q_sizes", C.c_void_p),
    ]


class NetOpts(C.Structure):
    _fields_ = [("min_space", C.c_int32), ("min_fill", C.c_int32), ("min_score", C.c_double),
                ("incl_hap", C.c_int32)]


class AxtInput(C.Structure):
    _fields_ = [("n_pairs", C.c_int64), ("t_seq", C.c_void_p), ("q_seq", C.c_void_p),
                ("q_strand", C.c_void_p), ("blk_off", C.c_void_p), ("blk_t", C.c_void_p),
                ("blk_q", C.c_void_p), ("blk_size", C.c_void_p)]


class AxtChains(C.Structure):
    _fields_ = [("n_chains", C.c_int64), ("score", C.POINTER(C.c_double)),
                ("pair", C.POINTER(C.c_int32)), ("t_start", C.POINTER(C.c_int32)),
                ("t_end", C.POINTER(C.c_int32)), ("q_start", C.POINTER(C.c_int32)),
                ("q_end", C.POINTER(C.c_int32)), ("blk_off", C.POINTER(C.c_int64)),
                ("n_blocks", C.c_int64), ("blk_t", C.POINTER(C.c_int32)),
                ("blk_q", C.POINTER(C.c_int32)), ("blk_size", C.POINTER(C.c_int32))]


# name -> (restype, argtypes)
_PROTOS = {
    "gac_abi_version": (C.c_int, []),
    "gac_last_error": (C.c_char_p, []),
    "gac_open": (C.c_int, [C.c_int, C.POINTER(C.c_void_p)]),
    "gac_close": (None, [C.c_void_p]),
    "gac_device_arch": (C.c_char_p, [C.c_void_p]),
    "gac_gapcalc_build": (C.c_int, [C.c_char_p, C.POINTER(C.POINTER(GapCalc))]),
    "gac_gapcalc_free": (None, [C.POINTER(GapCalc)]),
    "gac_scheme_read": (
        C.c_int,
        [C.c_char_p, C.POINTER(C.c_int32), C.POINTER(C.c_int32), C.POINTER(C.c_int32),
         C.POINTER(C.c_void_p)],
    ),
    "gac_gap_cost": (C.c_int, [C.POINTER(GapCalc), C.c_int, C.c_int]),
    "gac_set_scoring": (C.c_int, [C.c_void_p, C.POINTER(C.c_int32), C.POINTER(GapCalc)]),
    "gac_genome_load_2bit": (C.c_int, [C.c_void_p, C.c_int, C.c_char_p]),
    "gac_genome_add_seq": (
        C.c_int,
        [C.c_void_p, C.c_int, C.c_char_p, C.c_int32, C.c_void_p, C.c_int32, C.c_void_p,
         C.c_void_p],
    ),
    "gac_genome_finalize": (C.c_int, [C.c_void_p, C.c_int]),
    "gac_genome_seq_count": (C.c_int32, [C.c_void_p, C.c_int]),
    "gac_genome_seq_index": (C.c_int32, [C.c_void_p, C.c_int, C.c_char_p]),
    "gac_genome_seq_size": (C.c_int32, [C.c_void_p, C.c_int, C.c_int32]),
    "gac_genome_seq_name": (C.c_char_p, [C.c_void_p, C.c_int, C.c_int32]),
    "gac_genome_decode": (
        C.c_int, [C.c_void_p, C.c_int, C.c_int32, C.c_int32, C.c_int32, C.c_char_p]),
    "gac_chains_upload": (C.c_int, [C.c_void_p, C.POINTER(ChainsetDesc), C.POINTER(C.c_void_p)]),
    "gac_chains_reupload": (C.c_int, [C.c_void_p, C.POINTER(ChainsetDesc), C.c_void_p]),
    "gac_chains_free": (None, [C.c_void_p]),
    "gac_chains_context": (C.c_void_p, [C.c_void_p]),
    "gac_score_ranges_host": (C.c_int, [C.c_void_p, C.POINTER(ChainsetDesc), C.c_void_p, C.c_int64,
                                        C.c_uint32, C.c_void_p, C.c_void_p, C.c_void_p]),
    "gac_chains_block_count": (C.c_int64, [C.c_void_p]),
    "gac_score_ranges": (
        C.c_int,
        [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int64, C.c_uint32, C.c_void_p, C.c_void_p,
         C.c_void_p],
    ),
    "gac_score_ranges_device": (
        C.c_int,
        [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int64, C.c_uint32, C.c_void_p, C.c_void_p,
         C.c_void_p, C.c_void_p],
    ),
    "gac_score_windows": (
        C.c_int,
        [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int64, C.c_uint32, C.c_void_p, C.c_void_p,
         C.c_void_p],
    ),
    "gac_score_windows_device": (
        C.c_int,
        [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int64, C.c_uint32, C.c_void_p, C.c_void_p,
         C.c_void_p, C.c_void_p],
    ),
    "gac_score_chains": (
        C.c_int, [C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p, C.c_void_p]),
    "gac_score_chains_device": (
        C.c_int, [C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p, C.c_void_p,
                  C.c_void_p]),
    "gac_score_blocks": (
        C.c_int,
        [C.c_void_p, C.c_int64, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
         C.c_void_p, C.c_void_p, C.c_void_p],
    ),
    "gac_axt_chain": (
        C.c_int,
        [C.c_void_p, C.POINTER(C.c_int32), C.POINTER(GapCalc), C.POINTER(AxtInput), C.c_double,
         C.c_int, C.c_char_p, C.POINTER(C.POINTER(AxtChains))],
    ),
    "gac_axt_chains_free": (None, [C.POINTER(AxtChains)]),
    "gac_net_build": (C.c_int, [C.POINTER(NetInput), C.POINTER(NetOpts), C.POINTER(C.c_void_p)]),
    "gac_net_build_sides": (C.c_int, [C.POINTER(NetInput), C.POINTER(NetOpts), C.c_int,
                                      C.POINTER(C.c_void_p)]),
    "gac_net_build_subset": (C.c_int, [C.POINTER(NetInput), C.POINTER(NetOpts), C.c_void_p,
                                       C.c_void_p, C.POINTER(C.c_void_p)]),
    "gac_net_free": (None, [C.c_void_p]),
    "gac_net_netted": (C.c_int64, [C.c_void_p]),
    "gac_net_fill_count": (C.c_int64, [C.c_void_p, C.c_int]),
    "gac_net_get_fills": (
        C.c_int, [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]),
    "gac_net_get_fill_windows": (C.c_int, [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p]),
    "gac_net_rescore_windows": (C.c_int, [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p,
                                          C.c_void_p]),
    "gac_net_write": (
        C.c_int, [C.c_void_p, C.c_int, C.c_void_p, C.c_char_p, C.c_void_p, C.c_int32]),
    "gac_net_write_file": (
        C.c_int, [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int32]),
    "gac_net_write_begin": (
        C.c_int, [C.c_void_p, C.c_int, C.c_void_p, C.c_int32, C.POINTER(C.c_void_p)]),
    "gac_net_write_end": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p]),
    "gac_net_write_free": (None, [C.c_void_p]),
    "gac_chain_dp": (
        C.c_int, [C.c_void_p, C.c_int64] + [C.c_void_p] * 14),
    "gac_crossovers": (
        C.c_int, [C.c_void_p, C.c_int64] + [C.c_void_p] * 10),
    "gac_dev_alloc": (C.c_int, [C.c_void_p, C.c_size_t, C.POINTER(C.c_void_p)]),
    "gac_dev_free": (C.c_int, [C.c_void_p, C.c_void_p]),
    "gac_memcpy_h2d": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t]),
    "gac_memcpy_d2h": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t]),
    "gac_synchronize": (C.c_int, [C.c_void_p]),
    "gac_prof_enable": (C.c_int, [C.c_void_p, C.c_int]),
    "gac_prof_read": (C.c_int, [C.c_void_p, C.c_int, C.POINTER(C.c_double), C.POINTER(C.c_int64)]),
    "gac_prof_reset": (C.c_int, [C.c_void_p]),
    "gac_comm_open": (C.c_int, [C.c_char_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_double,
                                C.c_void_p, C.c_void_p, C.POINTER(C.c_void_p)]),
    "gac_comm_backend": (C.c_int, [C.c_void_p]),
    "gac_comm_init_seconds": (C.c_double, [C.c_void_p]),
    "gac_allgather": (C.c_int, [C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p]),
    "gac_allgatherv": (C.c_int, [C.c_void_p, C.c_void_p, C.c_size_t, C.POINTER(C.c_void_p),
                                 C.POINTER(C.c_size_t)]),
    "gac_comm_barrier": (C.c_int, [C.c_void_p]),
    "gac_comm_close": (None, [C.c_void_p]),
}

EXPORTED = tuple(_PROTOS)


def build(quiet: bool = True) -> None:
    """Build libgachain + tools in-tree with make (hipcc --offload-arch=gfx950)."""
    out = subprocess.run(
        ["make", "-C", REPO_DIR, "-j8", "all"],
        stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if out.returncode != 0:
        raise RuntimeError("building libgachain failed:\n" + out.stdout[-4000:])
    if not quiet:
        print(out.stdout)


def lib() -> C.CDLL:
    """Load libgachain.so (building it first if it is absent)."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            build()
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} missing: the HIP extension is required")
        L = C.CDLL(LIB_PATH)
        for name, (res, args) in _PROTOS.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        if L.gac_abi_version() != 1:
            raise RuntimeError("libgachain ABI mismatch")
        _lib = L
        return L


def check(rc: int) -> None:
    if rc != GAC_OK:
        msg = lib().gac_last_error()
        raise GacError(rc, msg.decode() if msg else "")
