"""gac_allgather's RCCL backend on the GPU (include/gachain.h): a one-rank
communicator (ncclGetUniqueId, ncclCommInitRank, ncclAllGather through HBM
on this process's device) and its set-up time; and the host backend between
two processes that both hold the same GPU (RCCL refuses two ranks on one
device, so that is the pairing a one-GPU box can run)."""
import ctypes as C
import os
import subprocess
import sys

import pytest

from conftest import REPO

pytestmark = pytest.mark.gpu

GAC_COMM_HOST, GAC_COMM_RCCL = 1, 2


def test_rccl_world1_allgather(tmp_path):
    from genomealignmenttools_amd import _lib
    L = _lib.lib()
    comm = C.c_void_p()
    _lib.check(L.gac_comm_open(str(tmp_path / "rv").encode(), 1, 0, 0, GAC_COMM_RCCL, 60.0, None,
                               None, C.byref(comm)))
    assert L.gac_comm_backend(comm) == GAC_COMM_RCCL
    init = L.gac_comm_init_seconds(comm)
    assert init > 0
    data = bytes(range(256)) * 64
    recv = C.create_string_buffer(len(data))
    _lib.check(L.gac_allgather(comm, data, len(data), recv))
    assert recv.raw == data
    p = C.c_void_p()
    counts = (C.c_size_t * 1)()
    _lib.check(L.gac_allgatherv(comm, data[:1000], 1000, C.byref(p), counts))
    assert counts[0] == 1000 and C.string_at(p, 1000) == data[:1000]
    C.CDLL(None).free(p)
    L.gac_comm_close(comm)
    print(f"RCCL communicator set-up {init * 1e3:.1f} ms")


WORKER = r"""
import ctypes as C, sys
sys.path.insert(0, {repo!r})
from genomealignmenttools_amd import _lib
L = _lib.lib()
ctx = C.c_void_p()
_lib.check(L.gac_open(0, C.byref(ctx)))           # both ranks hold GPU 0
comm = C.c_void_p()
r = int(sys.argv[2])
_lib.check(L.gac_comm_open(sys.argv[1].encode(), 2, r, 0, 1, 120.0, None, None, C.byref(comm)))
recv = C.create_string_buffer(8)
_lib.check(L.gac_allgather(comm, bytes([r]) * 4, 4, recv))
L.gac_comm_close(comm)
L.gac_close(ctx)
print(recv.raw.hex())
"""


def test_host_backend_two_ranks_one_gpu(tmp_path):
    script = tmp_path / "w.py"
    script.write_text(WORKER.format(repo=REPO))
    prefix = str(tmp_path / "rv2")
    procs = [subprocess.Popen([sys.executable, str(script), prefix, str(r)], stdout=subprocess.PIPE,
                              stderr=subprocess.PIPE, text=True) for r in range(2)]
    outs = []
    for p in procs:
        o, e = p.communicate(timeout=120)
        assert p.returncode == 0, e[-2000:]
        outs.append(o.strip())
    assert outs == ["0000000001010101"] * 2
