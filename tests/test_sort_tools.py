"""bin/chainSort and bin/chainMergeSort against the reference tools compiled
from /root/reference (oracle/_ref/chainSort, oracle/_ref/chainMergeSort;
kent/src/hg/mouseStuff/chainSort/chainSort.c:41-116,
kent/src/hg/mouseStuff/chainMergeSort/chainMergeSort.c:89-224): every output
byte-identical, on inputs with score ties, '#' lines at the top and between
chains, id-less headers, fractional scores, .gz input, -target / -query /
-index, -saveId, -inputList and the >400-file hierarchical merge.

The tools are host-only (no device); the same checks run in the CPU suite
and, marked gpu, in the GPU-box session."""
import filecmp
import gzip
import os
import subprocess

import numpy as np
import pytest

from conftest import GOLDEN


def _bin(name):
    from genomealignmenttools_amd._lib import BIN_DIR
    return os.path.join(BIN_DIR, name)


def _ref(name):
    from oracle.oracle import ref_tool
    p = ref_tool(name)
    if not os.path.exists(p):
        pytest.skip(f"{p} not built (needs /root/reference: make ref)")
    return p


def _chain_text(ca, idx, rng, frac=False, idless=False, meta_every=0):
    """chain records idx of ca as text; scores rounded to multiples of 500
    (ties), optionally fractional, optionally without the id field, with
    '#' lines between some chains."""
    out = []
    for k, i in enumerate(idx):
        if meta_every and k and k % meta_every == 0:
            out.append(f"# between chains {k}\n")
        sc = float(np.round(ca.score[i] / 500.0) * 500.0)
        if frac:
            sc += float(rng.choice([0.0, 0.25, 0.5, 0.75]))
        sc_txt = ("%1.2f" % sc) if frac else ("%1.0f" % sc)
        head = (f"chain {sc_txt} {ca.tname[i]} {ca.tsize[i]} + {ca.tstart[i]} {ca.tend[i]} "
                f"{ca.qname[i]} {ca.qsize[i]} {'-' if ca.qstrand[i] else '+'} {ca.qstart[i]} "
                f"{ca.qend[i]}")
        out.append(head + ("" if idless else f" {ca.id[i]}") + "\n")
        t, q, s = ca.blocks(int(i))
        for b in range(len(s) - 1):
            out.append(f"{s[b]}\t{t[b + 1] - t[b] - s[b]}\t{q[b + 1] - q[b] - s[b]}\n")
        out.append(f"{s[-1]}\n\n")
    return "".join(out)


@pytest.fixture(scope="module")
def chains():
    from genomealignmenttools_amd.chainfile import read_chains
    return read_chains(os.path.join(GOLDEN, "synth11", "in.chain"))


def _run(cmd, stdout=None, cwd=None):
    r = subprocess.run([str(c) for c in cmd], stdout=stdout or subprocess.PIPE,
                       stderr=subprocess.PIPE, cwd=cwd, timeout=300)
    assert r.returncode == 0, r.stderr.decode()[-2000:]
    return r


def check_chainsort(chains, tmp_path):
    rng = np.random.default_rng(5)
    idx = rng.permutation(chains.n)
    text = "# made for chainSort\n#second line\n" + _chain_text(chains, idx, rng, meta_every=37)
    (tmp_path / "in.chain").write_text(text)
    (tmp_path / "idless.chain").write_text(_chain_text(chains, idx[:120], rng, idless=True))
    with gzip.open(tmp_path / "in.chain.gz", "wt") as f:
        f.write(text)
    cases = [("in.chain", []), ("in.chain", ["-target"]), ("in.chain", ["-query"]),
             ("in.chain.gz", []), ("idless.chain", []), ("idless.chain", ["-query"])]
    for k, (inp, opts) in enumerate(cases):
        for tag in ("ours", "ref"):
            tool = _bin("chainSort") if tag == "ours" else _ref("chainSort")
            idx_opt = [f"-index={tmp_path}/{tag}{k}.idx"]
            _run([tool, tmp_path / inp, tmp_path / f"{tag}{k}.chain"] + opts)
            _run([tool, tmp_path / inp, tmp_path / f"{tag}{k}i.chain"] + opts + idx_opt)
        for suf in ("", "i"):
            assert filecmp.cmp(tmp_path / f"ours{k}{suf}.chain", tmp_path / f"ref{k}{suf}.chain",
                               shallow=False), (inp, opts, suf)
        assert filecmp.cmp(tmp_path / f"ours{k}.idx", tmp_path / f"ref{k}.idx", shallow=False)


def check_chainmergesort(chains, tmp_path, nfiles=12, frac=False, idless=False):
    """nfiles score-sorted inputs (the reference chainSort makes them; with
    idless, written sorted without header ids, so that chainIdNext numbers
    them in the merge's read order -- visible with -saveId) merged."""
    rng = np.random.default_rng(nfiles)
    parts = np.array_split(rng.permutation(chains.n), nfiles)
    names = []
    for k, p in enumerate(parts):
        srt = tmp_path / f"part{k}.chain"
        if idless:
            p = p[np.argsort(-np.round(chains.score[p] / 500.0), kind="stable")]
            srt.write_text(_chain_text(chains, p, rng, idless=True))
            names.append(str(srt))
            continue
        raw = tmp_path / f"raw{k}.chain"
        body = _chain_text(chains, p, rng, frac=frac, meta_every=11 if k % 3 == 0 else 0)
        raw.write_text((f"# part {k}\n" if k % 2 == 0 else "") + body)
        _run([_ref("chainSort"), raw, srt])
        if k % 4 == 1:  # a '#' line after the last chain
            with open(srt, "a") as f:
                f.write("# trailer\n")
        names.append(str(srt))
    (tmp_path / "list.txt").write_text("\n".join(names) + "\n")
    for opts in ([], ["-saveId"]):
        for tag in ("ours", "ref"):
            tool = _bin("chainMergeSort") if tag == "ours" else _ref("chainMergeSort")
            with open(tmp_path / f"{tag}.out", "wb") as f:
                _run([tool] + opts + names, stdout=f, cwd=tmp_path)
            with open(tmp_path / f"{tag}.list.out", "wb") as f:
                _run([tool, f"-inputList={tmp_path}/list.txt"] + opts, stdout=f, cwd=tmp_path)
        assert filecmp.cmp(tmp_path / "ours.out", tmp_path / "ref.out", shallow=False), opts
        assert filecmp.cmp(tmp_path / "ours.list.out", tmp_path / "ref.list.out",
                           shallow=False), opts


def test_chainsort_vs_reference(chains, tmp_path):
    check_chainsort(chains, tmp_path)


def test_chainmergesort_vs_reference(chains, tmp_path):
    check_chainmergesort(chains, tmp_path, nfiles=12)


def test_chainmergesort_idless_saveid_vs_reference(chains, tmp_path):
    """Inputs without header ids: -saveId shows the ids chainRead gave them,
    in the order the merge reads the files (interleaved, not file by file)."""
    check_chainmergesort(chains, tmp_path, nfiles=7, idless=True)


def test_chainmergesort_hierarchical_vs_reference(chains, tmp_path):
    """450 inputs (> MAXFILES = 400): the reference's two-level hierSort,
    with fractional scores whose ties appear only after the %1.0f round trip
    through its temp files."""
    check_chainmergesort(chains, tmp_path, nfiles=450, frac=True)


@pytest.mark.gpu
def test_sort_tools_gpu_session(chains, tmp_path):
    """The same checks in the GPU-box session (the tools are host-only)."""
    check_chainsort(chains, tmp_path)
    check_chainmergesort(chains, tmp_path, nfiles=450, frac=True)
