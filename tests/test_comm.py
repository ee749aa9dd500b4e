"""gac_allgather / gac_allgatherv (include/gachain.h) on CPU:
the host backend across 2 and 3 processes -- fixed and variable parts,
repeated calls, a barrier, nothing left beside the rendezvous prefix -- and
the errors a rank sees when a peer never arrives or fails.  The RCCL backend
needs a GPU per rank (tests/test_gpu_comm.py runs it at world 1 and the host
backend under the tools on one GPU)."""
import ctypes as C
import os
import subprocess
import sys

import pytest

from conftest import REPO

GAC_COMM_HOST = 1

WORKER = r"""
import ctypes as C, os, sys
sys.path.insert(0, {repo!r})
from genomealignmenttools_amd import _lib
L = _lib.lib()
prefix, n, r = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
comm = C.c_void_p()
_lib.check(L.gac_comm_open(prefix.encode(), n, r, -1, 1, 60.0, None, None, C.byref(comm)))
assert L.gac_comm_backend(comm) == 1
out = []
for call in range(3):
    mine = bytes([(r * 16 + call + k) % 251 for k in range(1000)])
    recv = C.create_string_buffer(1000 * n)
    _lib.check(L.gac_allgather(comm, mine, 1000, recv))
    out.append(recv.raw.hex())
    part = bytes([r + 1]) * (r * 7 + call)          # ragged, rank 0's empty on call 0
    p = C.c_void_p()
    counts = (C.c_size_t * n)()
    _lib.check(L.gac_allgatherv(comm, part, len(part), C.byref(p), counts))
    got = C.string_at(p, sum(counts)) if sum(counts) else b""
    C.CDLL(None).free(p)
    out.append(got.hex() + ":" + ",".join(str(c) for c in counts))
_lib.check(L.gac_comm_barrier(comm))
L.gac_comm_close(comm)
print("\n".join(out))
"""


def _run_world(tmp_path, n, env=None):
    prefix = str(tmp_path / "rv.gaccomm.tok1")
    script = tmp_path / "w.py"
    script.write_text(WORKER.format(repo=REPO))
    procs = [subprocess.Popen([sys.executable, str(script), prefix, str(n), str(r)],
                              stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                              env=dict(os.environ, **(env or {})))
             for r in range(n)]
    outs = []
    for p in procs:
        o, e = p.communicate(timeout=120)
        assert p.returncode == 0, e[-2000:]
        outs.append(o.split())
    return prefix, outs


@pytest.mark.parametrize("n", [2, 3])
def test_host_allgather_world(tmp_path, n):
    prefix, outs = _run_world(tmp_path, n)
    assert all(o == outs[0] for o in outs)  # every rank holds the same gathered bytes
    for call in range(3):
        want = b"".join(bytes([(r * 16 + call + k) % 251 for k in range(1000)]) for r in range(n))
        assert bytes.fromhex(outs[0][2 * call]) == want
        parts = [bytes([r + 1]) * (r * 7 + call) for r in range(n)]
        data, counts = outs[0][2 * call + 1].split(":")
        assert bytes.fromhex(data) == b"".join(parts)
        assert [int(c) for c in counts.split(",")] == [len(p) for p in parts]
    left = [f for f in os.listdir(tmp_path) if f.startswith(os.path.basename(prefix))]
    assert left == [], left


def test_world1_is_a_copy(tmp_path):
    from genomealignmenttools_amd import _lib
    L = _lib.lib()
    comm = C.c_void_p()
    _lib.check(L.gac_comm_open(str(tmp_path / "x").encode(), 1, 0, -1, GAC_COMM_HOST, 0.0, None,
                               None, C.byref(comm)))
    recv = C.create_string_buffer(5)
    _lib.check(L.gac_allgather(comm, b"abcde", 5, recv))
    assert recv.raw == b"abcde"
    L.gac_comm_close(comm)
    assert os.listdir(tmp_path) == []


def test_missing_peer_times_out_and_dead_peer_fails(tmp_path):
    from genomealignmenttools_amd import _lib
    L = _lib.lib()
    comm = C.c_void_p()
    _lib.check(L.gac_comm_open(str(tmp_path / "y").encode(), 2, 0, -1, GAC_COMM_HOST, 0.5, None,
                               None, C.byref(comm)))
    recv = C.create_string_buffer(8)
    rc = L.gac_allgather(comm, b"12345678", 8, recv)
    assert rc != 0 and b"after" in L.gac_last_error()
    L.gac_comm_close(comm)
    # a liveness callback naming rank 1 dead ends the wait at once
    ALIVE = C.CFUNCTYPE(C.c_int, C.c_int, C.c_void_p)
    dead = ALIVE(lambda rank, user: 0 if rank == 1 else 1)
    comm = C.c_void_p()
    _lib.check(L.gac_comm_open(str(tmp_path / "z").encode(), 2, 0, -1, GAC_COMM_HOST, 60.0,
                               C.cast(dead, C.c_void_p), None, C.byref(comm)))
    rc = L.gac_comm_barrier(comm)
    assert rc != 0 and b"peer rank 1 failed" in L.gac_last_error()
    L.gac_comm_close(comm)


def test_bad_arguments():
    from genomealignmenttools_amd import _lib
    L = _lib.lib()
    comm = C.c_void_p()
    assert L.gac_comm_open(b"/tmp/x", 2, 2, -1, GAC_COMM_HOST, 0.0, None, None, C.byref(comm)) != 0
    assert L.gac_comm_open(b"/tmp/x", 2, 0, -1, 2, 0.0, None, None, C.byref(comm)) != 0  # RCCL, no device
    assert L.gac_comm_open(b"", 1, 0, -1, GAC_COMM_HOST, 0.0, None, None, C.byref(comm)) != 0
