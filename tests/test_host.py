"""Host-side (CPU) checks of the product: the C ABI library loads and exports
every symbol include/gachain.h declares, host parsing matches the reference,
the netting engine and the chainNet tool reproduce the reference's .net files
byte for byte, and scoring fails loudly without a GPU (no CPU fallback)."""
import filecmp
import os
import re
import subprocess

import numpy as np
import pytest

from conftest import GOLDEN, REPO


def test_lib_exports_every_header_symbol():
    import ctypes
    from genomealignmenttools_amd import _lib
    hdr = open(os.path.join(REPO, "include", "gachain.h")).read()
    hdr = re.sub(r"/\*.*?\*/", "", hdr, flags=re.S)
    decl = set(re.findall(r"\b(gac_[a-z0-9_]+)\s*\(", hdr))
    assert len(decl) > 30
    L = ctypes.CDLL(_lib.LIB_PATH)
    missing = [s for s in sorted(decl) if not hasattr(L, s)]
    assert not missing, missing
    assert set(_lib.EXPORTED) <= decl


def test_host_threads_follow_cgroup_quota(tmp_path, monkeypatch):
    """An un-configured tool sizes its thread pools from the CPUs the process
    may use: the affinity mask, narrowed by the cgroup CPU quota (cpu.max,
    rounded up) -- not the host's online CPU count."""
    import ctypes
    from genomealignmenttools_amd import _lib
    L = ctypes.CDLL(_lib.LIB_PATH)
    affinity = len(os.sched_getaffinity(0))
    monkeypatch.delenv("GAC_THREADS", raising=False)
    monkeypatch.delenv("OMP_NUM_THREADS", raising=False)
    f = tmp_path / "cpu.max"
    for text, want in (("200000 100000\n", min(2, affinity)), ("150000 100000\n", min(2, affinity)),
                       ("50000 100000\n", 1), ("max 100000\n", affinity)):
        f.write_text(text)
        monkeypatch.setenv("GAC_CGROUP_CPU_MAX", str(f))
        assert L.gac_host_cpus() == want, text
        assert L.gac_host_threads() == min(want, 64), text
    monkeypatch.setenv("GAC_CGROUP_CPU_MAX", str(tmp_path / "absent"))
    assert L.gac_host_cpus() >= 1
    f.write_text("100000 100000\n")
    monkeypatch.setenv("GAC_CGROUP_CPU_MAX", str(f))
    monkeypatch.setenv("GAC_THREADS", "5")  # an explicit count wins
    assert L.gac_host_threads() == 5


def test_gapcalc_tables_match_oracle():
    from genomealignmenttools_amd.gachain import GapCosts
    from oracle.oracle import OracleGap
    for name in ["loose", "medium", os.path.join(GOLDEN, "linearGap.txt")]:
        t = GapCosts(name).tables()
        og = OracleGap(name)
        n = t["small_size"]
        assert t["q_small"][0] == 0
        assert list(t["q_small"][1:]) == [og.cost(i, 0) for i in range(1, n)]
        assert list(t["t_small"][1:]) == [og.cost(0, i) for i in range(1, n)]
        assert list(t["b_small"][2:]) == [og.cost(i // 2, i - i // 2) for i in range(2, n)]


def test_host_gap_cost_vs_reference():
    """gac_gap_cost (the host gapCalcCost axtChain's DP uses) against the
    reference's own gapCalcCost on 5.6k (dq, dt) shapes x 3 tables
    (tests/golden/gapcalc.json, generated with the reference objects)."""
    import json
    from genomealignmenttools_amd.gachain import GapCosts
    with open(os.path.join(GOLDEN, "gapcalc.json")) as f:
        d = json.load(f)
    for key, name in [("loose", "loose"), ("medium", "medium"),
                      ("file", os.path.join(GOLDEN, "linearGap.txt"))]:
        g = GapCosts(name)
        got = [g.cost(dq, dt) for dq, dt in d["pairs"]]
        assert got == d[key], key


def test_score_scheme_reader():
    from genomealignmenttools_amd.gachain import read_score_scheme
    m, go, ge, ex = read_score_scheme(os.path.join(GOLDEN, "c1", "HoxD55.q"))
    assert m.tolist() == [[91, -90, -25, -100], [-90, 100, -100, -25], [-25, -100, 100, -90],
                          [-100, -25, -90, 91]]
    assert (go, ge, ex) == (400, 30, "")
    m, go, ge, ex = read_score_scheme(os.path.join(GOLDEN, "chrM", "newStyleLastz.Q.txt"))
    assert m[0].tolist() == [79, -84, -55, -128] and m[2].tolist() == [-55, -174, 100, -84]
    # the reference writes this exact text as ##blastzParms (axt.c:869)
    assert ex == "bad_score=X:-1736,fill_score=-174,T=2,X=790,Y=4865,K=3000,L=3000"
    m, go, ge, ex = read_score_scheme(None)
    assert m[0].tolist() == [91, -114, -31, -123] and (go, ge) == (400, 30)


def test_chainfile_roundtrip(tmp_path):
    from genomealignmenttools_amd.chainfile import read_chains, write_chains
    src = os.path.join(GOLDEN, "synth11", "in.chain")
    ca = read_chains(src)
    out = tmp_path / "x.chain"
    write_chains(ca, str(out))
    body = [l for l in open(src) if not l.startswith("#")]
    assert open(out).read() == "".join(body)


def subset_windows(ca, chain, s, e):
    """chainSubsetOnT's window (kent/src/lib/chain.c:481-500) of each (chain,
    s, e): chain-local first block with tEnd > s, and the count of blocks from
    there with tStart < e."""
    first, cnt = np.zeros(len(chain), np.int64), np.zeros(len(chain), np.int64)
    for i, (c, a, b) in enumerate(zip(chain, s, e)):
        o0, o1 = ca.blk_off[c], ca.blk_off[c + 1]
        bt, bs = ca.blk_t[o0:o1], ca.blk_size[o0:o1]
        f = int(np.searchsorted(bt + bs, a, side="right"))
        k = f
        while k < len(bt) and bt[k] < b:
            k += 1
        first[i], cnt[i] = f, k - f
    return first, cnt


@pytest.mark.parametrize("case", ["synth11", "synth12", "zero_end", "c5", "split"])
def test_net_fill_windows(case, monkeypatch):
    """The window of every partial target fill, recorded by the netting while
    it makes the fill (gac_net_get_fill_windows, what chainNet -rescore hands
    gac_score_windows), is exactly chainSubsetOnT's window of the fill's final
    range -- including chains with zero-size blocks at their ends."""
    from genomealignmenttools_amd import synth
    from genomealignmenttools_amd._lib import GAC_T
    from genomealignmenttools_amd.chainfile import read_chains
    from genomealignmenttools_amd.chainnet import Net
    from genomealignmenttools_amd.synth import read_sizes
    if case.startswith("synth"):
        d = os.path.join(GOLDEN, case)
        ca = read_chains(os.path.join(d, "in.chain"))
        ts, qs = read_sizes(os.path.join(d, "t.sizes")), read_sizes(os.path.join(d, "q.sizes"))
    else:
        if case == "zero_end":
            tg, qg, ca = synth.small_case(seed=5, n_chains=300)
            ca = synth.zero_end_blocks(ca, every=2)
        elif case == "split":  # one big side netted in regions (chain slices: block offsets)
            monkeypatch.setenv("GAC_THREADS", "8")
            monkeypatch.setenv("GAC_TIMING", "1")
            tg, qg, ca = synth.small_case(seed=21, n_chains=30000, tsize=6_000_000,
                                          qsizes=(3_000_000, 2_000_000, 1_000_000), max_blocks=3000)
        else:
            tg, qg, ca = synth.c5_case(seed=3, n_chains=3000, scale=0.002, min_size=20_000)
        ts, qs = tg.sizes, qg.sizes
    for opts in ({}, {"min_space": 1}):
        net = Net(ca, ts, qs, 0.0, **opts)
        f = net.fills(GAC_T)
        part = (f["flags"] & 1) == 1
        assert part.sum() > 10
        first, cnt = subset_windows(ca, f["chain"][part], f["start"][part], f["end"][part])
        assert np.array_equal(f["first_block"][part], first)
        assert np.array_equal(f["n_blocks"][part], cnt)
        # chainNet -rescore's list in one pass: the partial printed fills
        sel = np.nonzero(f["flags"] == 3)[0]
        w, pos = net.rescore_windows()
        assert np.array_equal(pos, sel)
        want = np.stack([f["chain"][sel], f["start"][sel], f["end"][sel],
                         f["first_block"][sel], f["n_blocks"][sel]], 1)
        assert np.array_equal(w, want)
        net.close()


@pytest.mark.parametrize("seed", [11, 12])
def test_netting_engine_vs_reference(seed, tmp_path):
    """Plain chainNet (no -rescore: no GPU involved) through the Python
    binding of the netting engine and through the C tool."""
    from genomealignmenttools_amd._lib import BIN_DIR, GAC_Q, GAC_T
    from genomealignmenttools_amd.chainfile import read_chains
    from genomealignmenttools_amd.chainnet import Net
    from genomealignmenttools_amd.synth import read_sizes
    d = os.path.join(GOLDEN, f"synth{seed}")
    ca = read_chains(os.path.join(d, "in.chain"))
    net = Net(ca, read_sizes(os.path.join(d, "t.sizes")), read_sizes(os.path.join(d, "q.sizes")),
              2000)
    net.write(GAC_T, str(tmp_path / "t.net"), meta=ca.meta)
    net.write(GAC_Q, str(tmp_path / "q.net"), meta=ca.meta)
    assert filecmp.cmp(tmp_path / "t.net", os.path.join(d, "plain.t.net"), shallow=False)
    assert filecmp.cmp(tmp_path / "q.net", os.path.join(d, "plain.q.net"), shallow=False)
    r = subprocess.run([os.path.join(BIN_DIR, "chainNet"), os.path.join(d, "in.chain"),
                        os.path.join(d, "t.sizes"), os.path.join(d, "q.sizes"),
                        str(tmp_path / "t2.net"), str(tmp_path / "q2.net")],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    assert filecmp.cmp(tmp_path / "t2.net", os.path.join(d, "plain.t.net"), shallow=False)
    assert filecmp.cmp(tmp_path / "q2.net", os.path.join(d, "plain.q.net"), shallow=False)


def test_netting_target_side_only(tmp_path):
    """gac_net_build_sides with the target side only (chainCleaner's
    self-netting): the same target net; the query side refuses to write."""
    from genomealignmenttools_amd._lib import GAC_Q, GAC_T, GacError
    from genomealignmenttools_amd.chainfile import read_chains
    from genomealignmenttools_amd.chainnet import Net
    from genomealignmenttools_amd.synth import read_sizes
    d = os.path.join(GOLDEN, "synth12")
    ca = read_chains(os.path.join(d, "in.chain"))
    net = Net(ca, read_sizes(os.path.join(d, "t.sizes")), read_sizes(os.path.join(d, "q.sizes")),
              2000, sides=1 << GAC_T)
    net.write(GAC_T, str(tmp_path / "t.net"), meta=ca.meta)
    assert filecmp.cmp(tmp_path / "t.net", os.path.join(d, "plain.t.net"), shallow=False)
    with pytest.raises(GacError):
        net.write(GAC_Q, str(tmp_path / "q.net"), meta=ca.meta)


@pytest.mark.parametrize("seed", [11, 12])
@pytest.mark.parametrize("tag,opts", [("ms1", ["-minSpace=1", "-minScore=0"]),
                                      ("ms100", ["-minSpace=100", "-minFill=10"])])
def test_netting_options_vs_reference(seed, tag, opts, tmp_path):
    """chainNet space/fill/score thresholds (the space index's edge cases:
    1-bp spaces, spaces consumed whole) against the reference's nets
    (tests/golden/make_golden.py::net_variants)."""
    from genomealignmenttools_amd._lib import BIN_DIR
    d = os.path.join(GOLDEN, f"synth{seed}")
    r = subprocess.run([os.path.join(BIN_DIR, "chainNet"), os.path.join(d, "in.chain"),
                        os.path.join(d, "t.sizes"), os.path.join(d, "q.sizes"),
                        str(tmp_path / "t.net"), str(tmp_path / "q.net")] + opts,
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    assert filecmp.cmp(tmp_path / "t.net", os.path.join(d, f"{tag}.t.net"), shallow=False)
    assert filecmp.cmp(tmp_path / "q.net", os.path.join(d, f"{tag}.q.net"), shallow=False)


def test_tool_errors(tmp_path):
    """kent errAbort semantics: message on stderr, exit status 255."""
    from genomealignmenttools_amd._lib import BIN_DIR
    d = os.path.join(GOLDEN, "synth11")
    sc = os.path.join(BIN_DIR, "scoreChain")
    cn = os.path.join(BIN_DIR, "chainNet")
    r = subprocess.run([sc], capture_output=True, text=True)
    assert r.returncode == 255 and "usage" in r.stderr
    r = subprocess.run([sc, "a", "b", "c", "d", "-bogus"], capture_output=True, text=True)
    assert r.returncode == 255 and "-bogus is not a valid option" in r.stderr
    r = subprocess.run([sc, os.path.join(d, "in.chain"), os.path.join(d, "t.2bit"),
                        os.path.join(d, "q.2bit"), "/dev/null"], capture_output=True, text=True)
    assert r.returncode == 255 and "Must specify linear gap costs" in r.stderr
    r = subprocess.run([sc, os.path.join(d, "in.chain"), os.path.join(d, "t.2bit"),
                        os.path.join(d, "q.2bit"), "/dev/null", "-linearGap=loose",
                        "-returnOnlyScore", "-returnOnlyScoreAndCoords"], capture_output=True, text=True)
    assert r.returncode == 255 and "cannot specify both" in r.stderr
    # unsorted input
    lines = open(os.path.join(d, "in.chain")).read().split("\n\n")
    bad = tmp_path / "bad.chain"
    bad.write_text("\n\n".join([lines[1], lines[0]] + lines[2:]))
    r = subprocess.run([cn, str(bad), os.path.join(d, "t.sizes"), os.path.join(d, "q.sizes"),
                        "/dev/null", "/dev/null"], capture_output=True, text=True)
    assert r.returncode == 255 and "must be sorted in order of score" in r.stderr
    # sizes files that disagree with the chains (checked in parallel; the
    # first failing chain in file order reports, as chainNet.c does)
    qs = open(os.path.join(d, "q.sizes")).read()
    for name, text, msg in (("qbad", qs.replace("150000", "150001"),
                             "chrQ1 is 150000 in {c} but 150001 in {s}"),
                            ("qmiss", "".join(x for x in qs.splitlines(True) if "chrQ2" not in x),
                             "hashMustFindVal: 'chrQ2' not found")):
        sz = tmp_path / f"{name}.sizes"
        sz.write_text(text)
        ch = os.path.join(d, "in.chain")
        r = subprocess.run([cn, ch, os.path.join(d, "t.sizes"), str(sz), "/dev/null",
                            "/dev/null"], capture_output=True, text=True)
        assert r.returncode == 255 and msg.format(c=ch, s=sz) in r.stderr, r.stderr
    r = subprocess.run([cn, os.path.join(d, "in.chain"), os.path.join(d, "t.sizes"),
                        os.path.join(d, "q.sizes"), "/dev/null", "/dev/null", "-rescore"],
                       capture_output=True, text=True)
    assert r.returncode == 255 and "-tNibDir" in r.stderr


def test_chaincleaner_errors(tmp_path):
    """chainCleaner argument checks (errAbort, exit 255) -- all before any
    device work."""
    from genomealignmenttools_amd._lib import BIN_DIR
    cc = os.path.join(BIN_DIR, "chainCleaner")
    d = os.path.join(GOLDEN, "cleaner")
    p = lambda x: os.path.join(d, x)
    r = subprocess.run([cc], capture_output=True, text=True)
    assert r.returncode == 255 and "usage" in r.stderr and "-LRfoldThreshold" in r.stderr
    args = [p("in.chain"), p("t.2bit"), p("q.2bit"), str(tmp_path / "o.chain"),
            str(tmp_path / "o.bed")]
    r = subprocess.run([cc] + args + [f"-net={p('in.net')}"], capture_output=True, text=True)
    assert r.returncode == 255 and "Must specify linear gap costs" in r.stderr
    r = subprocess.run([cc] + args + ["-linearGap=loose"], capture_output=True, text=True)
    assert r.returncode == 255 and "You must specifiy -tSizes" in r.stderr
    r = subprocess.run([cc] + args + ["-linearGap=loose", f"-tSizes={p('t.sizes')}"],
                       capture_output=True, text=True)
    assert r.returncode == 255 and "You must specifiy -qSizes" in r.stderr
    r = subprocess.run([cc] + args + ["-linearGap=loose", "-LRfoldThreshold=x"],
                       capture_output=True, text=True)
    assert r.returncode == 255
    r = subprocess.run([cc, p("in.chain"), "/nonexistent.2bit", p("q.2bit"), "a", "b",
                        "-linearGap=loose"], capture_output=True, text=True)
    assert r.returncode == 255 and "does not exist" in r.stderr


def test_axtchain_errors(tmp_path):
    """axtChain argument and input checks (errAbort, exit 255) -- all before
    any device work."""
    from genomealignmenttools_amd._lib import BIN_DIR
    ax = os.path.join(BIN_DIR, "axtChain")
    d = os.path.join(GOLDEN, "chrM")
    r = subprocess.run([ax], capture_output=True, text=True)
    assert r.returncode == 255 and "usage" in r.stderr and "-minScore=N" in r.stderr
    args = [os.path.join(d, "newStyleLastz.psl"), os.path.join(d, "hg19.chrM.2bit"),
            os.path.join(d, "susScr3.chrM.2bit"), str(tmp_path / "o.chain")]
    r = subprocess.run([ax, "-psl"] + args, capture_output=True, text=True)
    assert r.returncode == 255 and "Must specify linear gap costs" in r.stderr
    r = subprocess.run([ax, "-psl", "-minScore=x", "-linearGap=loose"] + args,
                       capture_output=True, text=True)
    assert r.returncode == 255 and "not a valid integer" in r.stderr
    bad = tmp_path / "bad.psl"
    bad.write_text("#c\n1\t2\t3\n")
    r = subprocess.run([ax, "-psl", "-linearGap=loose", str(bad)] + args[1:],
                       capture_output=True, text=True)
    assert r.returncode == 255 and "is not a psLayout file" in r.stderr
    lines = open(os.path.join(d, "newStyleLastz.psl")).read().split("\n")
    body = [l for l in lines if l and not l.startswith("#")]
    w = body[0].split("\t")
    w[8] = "++"
    bad.write_text("\t".join(w) + "\n")
    r = subprocess.run([ax, "-psl", "-linearGap=loose", str(bad)] + args[1:],
                       capture_output=True, text=True)
    assert r.returncode == 255 and "requires PSLs to have implicit positive strand" in r.stderr


def test_axtchain_psl_errors_in_parallel_chunks(tmp_path):
    """A PSL big enough to be parsed in parallel chunks: the first bad line in
    file order is reported, with its file line number, whichever chunk a
    thread finishes first (lineFile semantics of a sequential read)."""
    from genomealignmenttools_amd._lib import BIN_DIR
    ax = os.path.join(BIN_DIR, "axtChain")
    d = os.path.join(GOLDEN, "chrM")
    lines = open(os.path.join(d, "newStyleLastz.psl")).read().split("\n")
    head = [l for l in lines if l.startswith("#")]
    body = [l for l in lines if l and not l.startswith("#")]
    rows = body * (6_000_000 // sum(len(b) + 1 for b in body) + 1)  # > 4 MB: many chunks
    n0 = len(head)
    bad_at, later = len(rows) // 3, 2 * len(rows) // 3
    w = rows[later].split("\t")
    rows[later] = "\t".join(w[:5])  # a later error of another kind
    rows[bad_at] = "\t".join(rows[bad_at].split("\t")[:20])  # 20 words
    psl = tmp_path / "big.psl"
    psl.write_text("\n".join(head + rows) + "\n")
    r = subprocess.run([ax, "-psl", "-linearGap=loose", str(psl), os.path.join(d, "hg19.chrM.2bit"),
                        os.path.join(d, "susScr3.chrM.2bit"), str(tmp_path / "o.chain")],
                       capture_output=True, text=True)
    assert r.returncode == 255
    assert f"Bad line {n0 + bad_at + 1} of {psl} wordCount is 20 instead of 21 or 23" in r.stderr


def test_no_cpu_fallback_without_gpu():
    """On a box without a usable gfx950 device every scoring entry point must
    fail loudly (there is no CPU path to fall back to)."""
    import torch
    from genomealignmenttools_amd import GacError
    from genomealignmenttools_amd.gachain import Engine
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(GacError, match="no CPU fallback"):
        Engine(0)


@pytest.mark.parametrize("net", ["synth11", "synth12q", "cleaner"])
@pytest.mark.parametrize("case", ["s3000", "two_sets", "eq", "batch"])
def test_netfilter_nonnested_vs_reference(net, case):
    """bin/NetFilterNonNested.perl (native, host only) byte-identical to the
    reference perl script on reference chainNet nets ("12" and batch modes)."""
    import json
    from genomealignmenttools_amd._lib import BIN_DIR
    d = os.path.join(GOLDEN, "netfilter")
    with open(os.path.join(d, "cases.json")) as f:
        opts = json.load(f)[case]
    r = subprocess.run([os.path.join(BIN_DIR, "NetFilterNonNested.perl"),
                        os.path.join(d, f"{net}.net")] + opts, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    assert r.stdout == open(os.path.join(d, f"{net}.{case}.out")).read()


@pytest.mark.parametrize("net", ["synth11", "cleaner", "big"])
@pytest.mark.parametrize("case", ["ucsc", "ucsc_keep", "scoref", "keep12", "keepbatch"])
def test_netfilter_typed_modes_vs_reference(net, case):
    """The synteny / score / keep-type modes (-doUCSCSynFilter,
    -doScoreFilter, -keepSyn/InvNetsWithScore; src/NetFilterNonNested.perl:
    268-396) on nets typed by the reference netSyntenic: byte-identical to
    the reference perl script (tests/golden/make_netfilter_golden.py)."""
    import json
    from genomealignmenttools_amd._lib import BIN_DIR
    d = os.path.join(GOLDEN, "netfilter")
    with open(os.path.join(d, "typed_cases.json")) as f:
        opts = json.load(f)[case]
    r = subprocess.run([os.path.join(BIN_DIR, "NetFilterNonNested.perl"),
                        os.path.join(d, f"{net}.syn.net")] + opts, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    assert r.stdout == open(os.path.join(d, f"{net}.syn.{case}.out")).read()


def test_netfilter_mode_errors():
    """The script's checks: -doScoreFilter needs -minScore1; the synteny modes
    need netSyntenic's type field; batch and "12" sets do not mix."""
    from genomealignmenttools_amd._lib import BIN_DIR
    tool = os.path.join(BIN_DIR, "NetFilterNonNested.perl")
    d = os.path.join(GOLDEN, "netfilter")
    r = subprocess.run([tool, os.path.join(d, "synth11.syn.net"), "-doScoreFilter"],
                       capture_output=True, text=True)
    assert r.returncode == 255 and "-minScore1 with -doScoreFilter" in r.stderr
    r = subprocess.run([tool, os.path.join(d, "synth11.net"), "-doUCSCSynFilter"],
                       capture_output=True, text=True)
    assert r.returncode == 255 and "cannot parse the net type" in r.stderr
    r = subprocess.run([tool, os.path.join(d, "synth11.syn.net"), "-doScoreFilter",
                        "-minScore1=40000"], capture_output=True, text=True)
    assert r.returncode == 255 and "No type field" in r.stderr  # the script's own quirk
    r = subprocess.run([tool, os.path.join(d, "synth11.net"), "-minScore1", "5", "-minScore", "3"],
                       capture_output=True, text=True)
    assert r.returncode == 255 and "BOTH batch filtering" in r.stderr


def _c5_small(tmp_path):
    from genomealignmenttools_amd import chainfile, synth
    tg, qg, ca = synth.c5_case(seed=77, n_chains=6000, scale=0.002, min_size=5000)
    d = str(tmp_path)
    synth.write_sizes(tg.sizes, os.path.join(d, "t.sizes"))
    synth.write_sizes(qg.sizes, os.path.join(d, "q.sizes"))
    with open(os.path.join(d, "in.chain"), "w") as f:
        f.write("# C5-shaped, seed 77\n")
        chainfile.write_chains(ca, f)
    return d


@pytest.mark.parametrize("nranks", [2, 5, 8])
def test_chainnet_ranks_vs_reference(nranks, tmp_path):
    """chainNet -nranks=N -rank=R (one process per rank; here without
    -rescore, so no device): every rank nets its share of the 455 + 66
    chromosome sides, rank 0 assembles the nets -- identical to the
    reference's single-process nets, '#' lines included."""
    from genomealignmenttools_amd._lib import BIN_DIR
    from oracle.oracle import have_ref, ref_tool
    d = _c5_small(tmp_path)
    p = lambda x: os.path.join(d, x)
    args = [p("in.chain"), p("t.sizes"), p("q.sizes")]
    procs = [subprocess.Popen([os.path.join(BIN_DIR, "chainNet")] + args +
                              [p("m.t.net"), p("m.q.net"), "-minScore=0", f"-nranks={nranks}",
                               f"-rank={r}"], stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                              env=dict(os.environ, GAC_RANK_TOKEN=f"t{nranks}"))
             for r in range(nranks)]
    for pr in procs:
        _, err = pr.communicate(timeout=120)
        assert pr.returncode == 0, err
    assert not [f for f in os.listdir(d) if ".gac" in f]  # no part or marker files left
    r = subprocess.run([os.path.join(BIN_DIR, "chainNet")] + args +
                       [p("one.t.net"), p("one.q.net"), "-minScore=0"], capture_output=True)
    assert r.returncode == 0
    assert filecmp.cmp(p("m.t.net"), p("one.t.net"), shallow=False)
    assert filecmp.cmp(p("m.q.net"), p("one.q.net"), shallow=False)
    assert open(p("m.t.net")).readline() == "# C5-shaped, seed 77\n"
    if have_ref():
        r = subprocess.run([ref_tool("chainNet")] + args + [p("ref.t.net"), p("ref.q.net"),
                                                           "-minScore=0"], capture_output=True)
        assert r.returncode == 0
        assert filecmp.cmp(p("m.t.net"), p("ref.t.net"), shallow=False)
        assert filecmp.cmp(p("m.q.net"), p("ref.q.net"), shallow=False)


def _ranks(tool, d, chain_of, n, token="tk", env=None, only=None):
    p = lambda x: os.path.join(d, x)
    e = dict(os.environ, GAC_RANK_TIMEOUT="600", **({"GAC_RANK_TOKEN": token} if token else {}),
             **(env or {}))
    return [subprocess.Popen([tool, p(chain_of(r)), p("t.sizes"), p("q.sizes"), p("m.t.net"),
                              p("m.q.net"), f"-nranks={n}", f"-rank={r}"],
                             stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, env=e)
            for r in (range(n) if only is None else only)]


def test_chainnet_ranks_failure(tmp_path):
    """A rank that fails makes every rank waiting on it fail too (errAbort
    status 255) within seconds -- not after GAC_RANK_TIMEOUT -- whichever rank
    it is, with no half-assembled output; bad -rank values and a missing run
    token are rejected."""
    import time
    from genomealignmenttools_amd._lib import BIN_DIR
    d = _c5_small(tmp_path)
    p = lambda x: os.path.join(d, x)
    with open(p("bad.chain"), "w") as f:
        f.write("chain 10 chr1 5 + 0 1\n")
    tool = os.path.join(BIN_DIR, "chainNet")
    for n, bad in ((2, 1), (3, 1), (3, 0), (4, 2)):
        t0 = time.time()
        procs = _ranks(tool, d, lambda r: "bad.chain" if r == bad else "in.chain", n,
                       token=f"f{n}{bad}")
        outs = [pr.communicate(timeout=120) for pr in procs]
        assert time.time() - t0 < 60, (n, bad)
        # the failing rank, rank 0 and every rank placed after it fail; ranks
        # between 0 and it need only rank 0's sizes and may finish
        for r in range(n):
            if r == 0 or r >= bad:
                assert procs[r].returncode == 255, (n, bad, r, outs[r][1][-300:])
            if r != bad and procs[r].returncode == 255:
                assert "failed" in outs[r][1], outs[r][1]
    r = subprocess.run([tool, p("in.chain"), p("t.sizes"), p("q.sizes"), "a", "b", "-nranks=2",
                        "-rank=2"], capture_output=True, text=True,
                       env=dict(os.environ, GAC_RANK_TOKEN="x"))
    assert r.returncode == 255 and "-rank=2" in r.stderr
    env = {k: v for k, v in os.environ.items() if k != "GAC_RANK_TOKEN"}
    r = subprocess.run([tool, p("in.chain"), p("t.sizes"), p("q.sizes"), "a", "b", "-nranks=2",
                        "-rank=0"], capture_output=True, text=True, env=env)
    assert r.returncode == 255 and "GAC_RANK_TOKEN" in r.stderr


def test_chainnet_ranks_killed(tmp_path):
    """A rank killed outright (SIGKILL: no failure marker) is noticed by the
    ranks waiting on it through its liveness file: they exit 255 within
    seconds instead of waiting GAC_RANK_TIMEOUT; a rank that never starts
    ends the wait after GAC_RANK_START_TIMEOUT."""
    import signal
    import time
    from genomealignmenttools_amd._lib import BIN_DIR
    d = _c5_small(tmp_path)
    p = lambda x: os.path.join(d, x)
    os.mkfifo(p("stall.chain"))  # rank 1 blocks opening it, after publishing its liveness
    tool = os.path.join(BIN_DIR, "chainNet")
    procs = _ranks(tool, d, lambda r: "stall.chain" if r == 1 else "in.chain", 3, token="kill3")
    alive = p("m.t.net.gacpart1.kill3.alive")
    t0 = time.time()
    while not os.path.exists(alive) and time.time() - t0 < 60:
        time.sleep(0.05)
    assert os.path.exists(alive)
    time.sleep(0.5)
    procs[1].send_signal(signal.SIGKILL)
    t0 = time.time()
    outs = [pr.communicate(timeout=120) for pr in procs]
    assert time.time() - t0 < 30
    assert procs[1].returncode == -signal.SIGKILL
    for r in (0, 2):
        assert procs[r].returncode == 255 and "rank 1 died" in outs[r][1], outs[r][1]
    # rank 2 never launched: ranks 0 and 1 give up after the start timeout
    t0 = time.time()
    procs = _ranks(tool, d, lambda r: "in.chain", 3, token="nostart",
                   env={"GAC_RANK_START_TIMEOUT": "3"}, only=(0, 1))
    outs = [pr.communicate(timeout=120) for pr in procs]
    assert time.time() - t0 < 60
    assert procs[0].returncode == 255 and "did not start" in outs[0][1], outs[0][1]


@pytest.mark.parametrize("opts", [["-minScore=0"], ["-minSpace=1", "-minScore=0"],
                                  ["-minSpace=300", "-minFill=40"]])
def test_netting_split_side_vs_reference(opts, tmp_path):
    """One big chromosome side netted by many threads (gac_net.c net_regions:
    a short sequential prefix, then regions between space boundaries):
    identical to the sequential engine (GAC_NET_SPLIT=0) and to the
    reference chainNet."""
    from genomealignmenttools_amd import chainfile, synth
    from genomealignmenttools_amd._lib import BIN_DIR
    from oracle.oracle import have_ref, ref_tool
    tg, qg, ca = synth.small_case(seed=21, n_chains=30000, tsize=6_000_000,
                                  qsizes=(3_000_000, 2_000_000, 1_000_000), max_blocks=3000)
    d = str(tmp_path)
    p = lambda x: os.path.join(d, x)
    synth.write_sizes(tg.sizes, p("t.sizes"))
    synth.write_sizes(qg.sizes, p("q.sizes"))
    chainfile.write_chains(ca, p("in.chain"))
    args = [p("in.chain"), p("t.sizes"), p("q.sizes")]
    outs = {}
    for tag, env in (("split", {"GAC_THREADS": "8", "GAC_TIMING": "1"}),
                     ("seq", {"GAC_THREADS": "8", "GAC_NET_SPLIT": "0"})):
        r = subprocess.run([os.path.join(BIN_DIR, "chainNet")] + args +
                           [p(f"{tag}.t.net"), p(f"{tag}.q.net")] + opts,
                           capture_output=True, text=True, env=dict(os.environ, **env))
        assert r.returncode == 0, r.stderr
        outs[tag] = r.stderr
    assert "regions" in outs["split"]  # the target side was split
    for side in "tq":
        assert filecmp.cmp(p(f"split.{side}.net"), p(f"seq.{side}.net"), shallow=False)
    if have_ref():
        r = subprocess.run([ref_tool("chainNet")] + args + [p("ref.t.net"), p("ref.q.net")] + opts,
                           capture_output=True)
        assert r.returncode == 0
        for side in "tq":
            assert filecmp.cmp(p(f"split.{side}.net"), p(f"ref.{side}.net"), shallow=False)


def test_kent_shim_library_exports_and_gapcalc():
    """libgachain_kent.so exports every function include/gachain_kent.h
    declares, and its gapCalcCost equals the reference's on the golden gap
    shapes (gapCalc.c:298-331; no device involved)."""
    import ctypes as C
    import json
    import re
    from genomealignmenttools_amd._lib import LIB_DIR
    hdr = open(os.path.join(REPO, "include", "gachain_kent.h")).read()
    hdr = re.sub(r"/\*.*?\*/", "", hdr, flags=re.S)  # comments out
    hdr = re.sub(r"^\s*#.*$", "", hdr, flags=re.M)  # preprocessor lines out
    hdr = re.sub(r"\{[^{}]*\}", "", hdr)  # struct bodies out
    hdr = re.sub(r"\btypedef\b[^;]*;", "", hdr)  # typedefs out
    decl = set(re.findall(r"\b(\w+)\s*\([^;{]*\)\s*;", hdr)) - {"if", "sizeof"}
    assert {"chainCalcScore", "chainSubsetOnT", "gapCalcCost", "gac_kent_bind"} <= decl
    lib = C.CDLL(os.path.join(LIB_DIR, "libgachain_kent.so"))
    for name in decl:
        assert hasattr(lib, name), name
    lib.gapCalcFromFile.restype = C.c_void_p
    lib.gapCalcFromFile.argtypes = [C.c_char_p]
    lib.gapCalcCost.argtypes = [C.c_void_p, C.c_int, C.c_int]
    with open(os.path.join(GOLDEN, "gapcalc.json")) as f:
        gj = json.load(f)
    pairs = gj["pairs"][:2000]
    for name, src in [("loose", b"loose"), ("medium", b"medium"),
                      ("file", os.path.join(GOLDEN, "linearGap.txt").encode())]:
        gc = lib.gapCalcFromFile(src)
        got = [lib.gapCalcCost(gc, int(dq), int(dt)) for dq, dt in pairs]
        assert got == gj[name][:2000], name


def test_net_write_two_phase(tmp_path):
    """gac_net_write_begin/_end (chainNet -rescore formats the target net
    while the GPU rescores): the same bytes as gac_net_write with the same
    scores, rescored scores <= 0 printed as 1; with minScore > 1 the two-phase
    writer refuses (which fills print would depend on the scores)."""
    import ctypes as C
    from genomealignmenttools_amd import chainfile
    from genomealignmenttools_amd._lib import lib
    from genomealignmenttools_amd.chainnet import Net as NetBuilder
    from genomealignmenttools_amd.synth import read_sizes
    d = os.path.join(GOLDEN, "synth11")
    ca = chainfile.read_chains(os.path.join(d, "in.chain"))
    ts, qs = read_sizes(os.path.join(d, "t.sizes")), read_sizes(os.path.join(d, "q.sizes"))
    libc = C.CDLL(None)
    libc.fopen.restype = C.c_void_p
    libc.fopen.argtypes = [C.c_char_p, C.c_char_p]
    libc.fclose.argtypes = [C.c_void_p]
    for min_score in (0.0, 1.0):
        nb = NetBuilder(ca, ts, qs, min_score=min_score)
        nf = lib().gac_net_fill_count(nb.h, 0)
        rng = np.random.default_rng(5)
        scores = rng.integers(-50, 10 ** 7, nf).astype(np.int64)
        scores[::7] = 0
        meta = ["# two-phase test"]
        nb.write(0, str(tmp_path / "a.net"), scores, meta)
        marr = (C.c_char_p * 1)(meta[0].encode())
        h = C.c_void_p()
        assert lib().gac_net_write_begin(nb.h, 0, C.cast(marr, C.c_void_p), 1, C.byref(h)) == 0
        f = libc.fopen(str(tmp_path / "b.net").encode(), b"w")
        assert lib().gac_net_write_end(h, scores.ctypes.data, f) == 0
        assert libc.fclose(f) == 0
        assert filecmp.cmp(tmp_path / "a.net", tmp_path / "b.net", shallow=False)
        nb.close()
    nb = NetBuilder(ca, ts, qs, min_score=2000.0)
    h = C.c_void_p()
    assert lib().gac_net_write_begin(nb.h, 0, None, 0, C.byref(h)) != 0
    nb.close()


def _hap_case(d):
    """A small set whose query names include haplotype/alt sequences."""
    from genomealignmenttools_amd import chainfile, synth
    tg, qg, ca = synth.small_case(seed=21, n_chains=300)
    ren = {"chrQ2": "chrQ2_hap1", "chrQ3": "chrQ3_alt"}
    qsizes = {ren.get(k, k): v for k, v in qg.sizes.items()}
    ca.qname = [ren.get(n, n) for n in ca.qname]
    synth.write_sizes(tg.sizes, os.path.join(d, "t.sizes"))
    synth.write_sizes(qsizes, os.path.join(d, "q.sizes"))
    chainfile.write_chains(ca, os.path.join(d, "in.chain"))


@pytest.mark.parametrize("mode", ["plain", "inclHap", "gz", "stdin"])
def test_chainnet_input_modes_vs_reference(mode, tmp_path):
    """chainNet's haplotype filter (`_hap`/`_alt` query names skipped unless
    -inclHap, chainNet.c:253-257), a .gz chain file (read through gzip like
    lineFileOpen) and `stdin` as the chain file name, against the reference
    chainNet (oracle/_ref) on the same input.  Plain netting: no device."""
    import gzip
    import shutil
    from genomealignmenttools_amd._lib import BIN_DIR
    from oracle.oracle import ref_tool
    ref = ref_tool("chainNet")
    if not os.path.exists(ref):
        pytest.skip("oracle/_ref/chainNet not built (make ref)")
    d = str(tmp_path)
    _hap_case(d)
    p = lambda x: os.path.join(d, x)
    chain = p("in.chain")
    opts = ["-inclHap"] if mode == "inclHap" else []
    if mode == "gz":
        with open(chain, "rb") as f, gzip.open(p("in.chain.gz"), "wb") as g:
            shutil.copyfileobj(f, g)
        chain = p("in.chain.gz")
    outs = {}
    for tag, exe in (("ours", os.path.join(BIN_DIR, "chainNet")), ("ref", ref)):
        src = "stdin" if mode == "stdin" else chain
        with open(p("in.chain"), "rb") as fin:
            r = subprocess.run([exe, src, p("t.sizes"), p("q.sizes"), p(f"{tag}.t.net"),
                                p(f"{tag}.q.net")] + opts,
                               stdin=fin if mode == "stdin" else None, capture_output=True)
        assert r.returncode == 0, r.stderr[-2000:]
        outs[tag] = [open(p(f"{tag}.{s}.net"), "rb").read() for s in "tq"]
    assert outs["ours"] == outs["ref"]
    qnet = outs["ours"][1].decode()
    if mode == "inclHap":
        assert "chrQ2_hap1" in qnet
    else:  # the haplotype query sides are netted only with -inclHap
        assert "net chrQ2_hap1" not in qnet


@pytest.mark.parametrize("tool", ["chainNet", "chainSort"])
def test_mapped_output_path(tool, tmp_path):
    """The large-output path of gac_par_output (every run formatted, then
    copied into a shared mapping of the reserved file range by all threads),
    forced on small files with GAC_OUTPUT_MMAP_MIN=0: same bytes as the
    reference's goldens, header lines before the mapped range included."""
    from genomealignmenttools_amd._lib import BIN_DIR
    d = os.path.join(GOLDEN, "synth11")
    env = dict(os.environ, GAC_OUTPUT_MMAP_MIN="0")
    if tool == "chainNet":
        r = subprocess.run([os.path.join(BIN_DIR, "chainNet"), os.path.join(d, "in.chain"),
                            os.path.join(d, "t.sizes"), os.path.join(d, "q.sizes"),
                            str(tmp_path / "t.net"), str(tmp_path / "q.net")],
                           capture_output=True, text=True, env=env)
        assert r.returncode == 0, r.stderr
        assert filecmp.cmp(tmp_path / "t.net", os.path.join(d, "plain.t.net"), shallow=False)
        assert filecmp.cmp(tmp_path / "q.net", os.path.join(d, "plain.q.net"), shallow=False)
    else:
        outs = {}
        for tag, e in (("mapped", env), ("plain", dict(os.environ, GAC_OUTPUT_MMAP_MIN="-1"))):
            r = subprocess.run([os.path.join(BIN_DIR, "chainSort"), os.path.join(d, "in.chain"),
                                str(tmp_path / f"{tag}.chain")], capture_output=True, text=True,
                               env=e)
            assert r.returncode == 0, r.stderr
            outs[tag] = open(tmp_path / f"{tag}.chain", "rb").read()
        assert outs["mapped"] == outs["plain"] and len(outs["plain"]) > 0


def test_write_chains_fast_negative_fields(tmp_path):
    """write_chains_fast sizes '-' signs of header integers (a negative id is
    legal input): the same bytes as write_chains."""
    from genomealignmenttools_amd import chainfile
    from genomealignmenttools_amd.chainfile import ChainArrays
    ca = ChainArrays(score=np.array([5.0, -3.0]), tname=["chr1", "chr2"],
                     tsize=np.array([1000, 900], np.int32), tstart=np.array([10, 20], np.int32),
                     tend=np.array([60, 70], np.int32), qname=["q1", "q2"],
                     qsize=np.array([800, 700], np.int32), qstrand=np.array([0, 1], np.uint8),
                     qstart=np.array([5, 6], np.int32), qend=np.array([55, 56], np.int32),
                     id=np.array([-7, 3], np.int64), blk_off=np.array([0, 2, 3], np.int64),
                     blk_t=np.array([10, 40, 20], np.int32), blk_q=np.array([5, 35, 6], np.int32),
                     blk_size=np.array([20, 20, 50], np.int32))
    chainfile.write_chains(ca, str(tmp_path / "a"))
    chainfile.write_chains_fast(ca, str(tmp_path / "b"))
    assert (tmp_path / "a").read_bytes() == (tmp_path / "b").read_bytes()


@pytest.mark.parametrize("opts", [[], ["-minSpace=1", "-minFill=1"]])
def test_chainnet_zero_size_blocks_vs_reference(opts, tmp_path):
    """Zero-size blocks (inside a chain's gaps, and as a chain's first
    block) against the reference chainNet: innerBounds counts them, the
    fill's final bounds and other-side range (rCalcOtherFill) keep them only
    strictly inside the fill -- the path add_chain_side takes a second walk
    over the blocks for.  (With -minFill=0 the reference asserts on the
    zero-size fills such blocks make, fillSpace's `s < e`: no case here.)"""
    from genomealignmenttools_amd import chainfile, synth
    from genomealignmenttools_amd._lib import BIN_DIR
    from oracle.oracle import ref_tool
    ref = ref_tool("chainNet")
    if not os.path.exists(ref):
        pytest.skip("oracle/_ref/chainNet not built (make ref)")
    tg, qg, ca = synth.small_case(seed=23, n_chains=300)
    bt, bq, bs, off = [], [], [], [0]
    for i in range(ca.n):
        t, q, z = (x.tolist() for x in ca.blocks(i))
        nt, nq, nz = [], [], []
        for k in range(len(t)):
            if k == 0 and i % 3 == 0 and t[0] > 0 and q[0] > 0:  # a zero-size first block
                nt.append(t[0] - 1), nq.append(q[0] - 1), nz.append(0)
            nt.append(t[k]), nq.append(q[k]), nz.append(z[k])
            if k + 1 < len(t) and i % 2 == 0:  # one inside the gap, when there is room
                gt, gq = t[k + 1] - (t[k] + z[k]), q[k + 1] - (q[k] + z[k])
                if gt >= 2 and gq >= 2:
                    nt.append(t[k] + z[k] + gt // 2), nq.append(q[k] + z[k] + gq // 2), nz.append(0)
        bt += nt
        bq += nq
        bs += nz
        off.append(off[-1] + len(nt))
        ca.tstart[i], ca.qstart[i] = nt[0], nq[0]
    ca.blk_t = np.array(bt, np.int32)
    ca.blk_q = np.array(bq, np.int32)
    ca.blk_size = np.array(bs, np.int32)
    ca.blk_off = np.array(off, np.int64)
    d = str(tmp_path)
    p = lambda x: os.path.join(d, x)
    synth.write_sizes(tg.sizes, p("t.sizes"))
    synth.write_sizes(qg.sizes, p("q.sizes"))
    chainfile.write_chains(ca, p("in.chain"))
    outs = {}
    for tag, exe in (("ours", os.path.join(BIN_DIR, "chainNet")), ("ref", ref)):
        r = subprocess.run([exe, p("in.chain"), p("t.sizes"), p("q.sizes"), p(f"{tag}.t.net"),
                            p(f"{tag}.q.net")] + opts, capture_output=True)
        assert r.returncode == 0, r.stderr[-2000:]
        outs[tag] = [open(p(f"{tag}.{s}.net"), "rb").read() for s in "tq"]
    assert outs["ours"] == outs["ref"]
