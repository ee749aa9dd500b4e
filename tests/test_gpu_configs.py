"""GPU parity at the BASELINE configs' shapes, the reference run in the same
test as the checker (C2, C3, C4, C5).

Every test generates its seeded synthetic input (genomes written as .2bit,
chains/PSL as text), runs the drop-in tool (bin/<tool>, HIP path) and the
reference tool compiled from /root/reference by oracle/ref.mk
(oracle/_ref/<tool>, test infrastructure) on the same files, and compares
every output byte for byte.  Sizes are chosen so that the reference finishes
in about a minute on the GPU box's host.

  C5:        all 455 hg38 x 66 mm10 sequences at their real lengths
             (gac_synth, the bench's generator), 400k chains, 9.1 M blocks,
             364 M aligned bases: scoreChain (two output modes, -nranks 2/3)
             + chainNet -rescore (also sparse upload, -nranks 2/3)
  C2:        hg38 chr1 x all mm10 at full length, 200k chains:
             chainNet -rescore
  C3:        C2 + 1000 planted chain-breaking-alignment loci on chr1:
             chainCleaner -net= (about 12.5k suspects removed)
  C4-shaped: 24 x 21 chromosome pairs x 2 strands, power-law blocks per
             pair, 1.2 M PSL blocks (host and device DP) and 5 M PSL blocks
             (the default hybrid DP, and the device DP alone): axtChain -psl
plus the edge cases the round-1 review listed: a custom -linearGap file on
the device, zero-size terminal blocks, chainNet -rescore's subset-upload
branch (a sequence missing from the 2bit), no partial fills at all, and a
clean exit status on failures while helper threads are live.
"""
import filecmp
import json
import os
import re
import subprocess

import numpy as np
import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu


def _bin(name):
    from genomealignmenttools_amd._lib import BIN_DIR
    return os.path.join(BIN_DIR, name)


def _ref(name):
    from oracle.oracle import ref_tool
    p = ref_tool(name)
    if not os.path.exists(p):
        pytest.fail(f"reference tool {p} not built (make ref)")
    return p


def _run(cmd, cwd=None, rc=0, timeout=900, env=None):
    r = subprocess.run([str(c) for c in cmd], capture_output=True, text=True, timeout=timeout,
                       cwd=cwd, env=dict(os.environ, **env) if env else None)
    assert r.returncode == rc, (cmd[0], r.returncode, r.stderr[-2000:])
    return r


def _same(a, b):
    assert filecmp.cmp(a, b, shallow=False), f"{a} differs from {b}"


def _write_case(d, tg, qg, ca):
    from genomealignmenttools_amd import chainfile, synth
    synth.write_2bit(tg, os.path.join(d, "t.2bit"))
    synth.write_2bit(qg, os.path.join(d, "q.2bit"))
    synth.write_sizes(tg.sizes, os.path.join(d, "t.sizes"))
    synth.write_sizes(qg.sizes, os.path.join(d, "q.sizes"))
    chainfile.write_chains(ca, os.path.join(d, "in.chain"))


def _rescore_pair(d, tag, extra=()):
    """bin/chainNet and oracle/_ref/chainNet -rescore on d/in.chain."""
    p = lambda x: os.path.join(d, x)
    opts = ["-rescore", f"-tNibDir={p('t.2bit')}", f"-qNibDir={p('q.2bit')}"] + list(extra)
    if not any(o.startswith("-linearGap=") for o in opts):
        opts.append("-linearGap=loose")
    args = [p("in.chain"), p("t.sizes"), p("q.sizes")]
    _run([_bin("chainNet")] + args + [p(f"{tag}.ours.t.net"), p(f"{tag}.ours.q.net")] + opts)
    _run([_ref("chainNet")] + args + [p(f"{tag}.ref.t.net"), p(f"{tag}.ref.q.net")] + opts)
    _same(p(f"{tag}.ours.t.net"), p(f"{tag}.ref.t.net"))
    _same(p(f"{tag}.ours.q.net"), p(f"{tag}.ref.q.net"))


# ---------------------------------------------------------------- C5
@pytest.fixture(scope="module")
def c5_dir(tmp_path_factory):
    """C5 at full genome lengths by gac_synth (csrc/synth/gac_synth.c, built
    by `make synth`), 400k chains."""
    from genomealignmenttools_amd._lib import PKG_DIR
    d = str(tmp_path_factory.mktemp("c5"))
    _run([os.path.join(PKG_DIR, "libexec", "gac_synth"), "c5", d, "-seed=1234",
          "-chains=400000", f"-sizesDir={os.path.join(PKG_DIR, 'data')}", "-threads=16"])
    with open(os.path.join(d, "info.json")) as f:
        info = json.load(f)
    assert info["t_seqs"] == 455 and info["q_seqs"] == 66 and info["scale"] == 1
    assert info["blocks"] > 8_000_000
    return d


@pytest.mark.timeout(900)
@pytest.mark.parametrize("nranks", [2, 3])
def test_c5_shaped_scorechain_ranks(c5_dir, nranks):
    """scoreChain -nranks=N -rank=R (one process per rank; all on device 0
    here): each rank scores a contiguous share of the chains, rank 0 writes
    the file -- identical to the reference's single run."""
    p = lambda x: os.path.join(c5_dir, x)
    args = [p("in.chain"), p("t.2bit"), p("q.2bit")]
    if not os.path.exists(p("sc.chain.ref")):
        _run([_ref("scoreChain")] + args + [p("sc.chain.ref"), "-linearGap=loose"])
    out = p(f"sc.ranks{nranks}")
    procs = [subprocess.Popen([_bin("scoreChain")] + args + [out, "-linearGap=loose",
                                                            f"-nranks={nranks}", f"-rank={r}",
                                                            "-gpu=0"],
                              stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                              env=dict(os.environ, GAC_RANK_TOKEN=f"sc{nranks}"))
             for r in range(nranks)]
    for r, pr in enumerate(procs):
        _, err = pr.communicate(timeout=600)
        assert pr.returncode == 0, (r, err[-2000:])
    _same(out, p("sc.chain.ref"))
    assert not [f for f in os.listdir(c5_dir) if ".gacpart" in f]


@pytest.mark.timeout(900)
@pytest.mark.parametrize("mode", ["chain", "coords"])
def test_c5_shaped_scorechain(c5_dir, mode):
    p = lambda x: os.path.join(c5_dir, x)
    args = [p("in.chain"), p("t.2bit"), p("q.2bit")]
    flag = ["-returnOnlyScoreAndCoords"] if mode == "coords" else []
    _run([_bin("scoreChain")] + args + [p(f"sc.{mode}.ours"), "-linearGap=loose"] + flag)
    _run([_ref("scoreChain")] + args + [p(f"sc.{mode}.ref"), "-linearGap=loose"] + flag)
    _same(p(f"sc.{mode}.ours"), p(f"sc.{mode}.ref"))


@pytest.fixture(scope="module")
def c5_ref_nets(c5_dir):
    """The reference chainNet -rescore nets of the C5-shaped set (run once)."""
    p = lambda x: os.path.join(c5_dir, x)
    _run([_ref("chainNet"), p("in.chain"), p("t.sizes"), p("q.sizes"), p("ref.t.net"),
          p("ref.q.net"), "-rescore", f"-tNibDir={p('t.2bit')}", f"-qNibDir={p('q.2bit')}",
          "-linearGap=loose"])
    return p("ref.t.net"), p("ref.q.net")


@pytest.mark.timeout(900)
def test_c5_shaped_chainnet_rescore(c5_dir, c5_ref_nets):
    p = lambda x: os.path.join(c5_dir, x)
    _run([_bin("chainNet"), p("in.chain"), p("t.sizes"), p("q.sizes"), p("c5.t.net"),
          p("c5.q.net"), "-rescore", f"-tNibDir={p('t.2bit')}", f"-qNibDir={p('q.2bit')}",
          "-linearGap=loose"])
    _same(p("c5.t.net"), c5_ref_nets[0])
    _same(p("c5.q.net"), c5_ref_nets[1])


@pytest.mark.timeout(900)
def test_c5_shaped_chainnet_rescore_sparse(c5_dir, c5_ref_nets):
    """GAC_NET_SPARSE=1: only the genome words under the chains' blocks go
    to HBM (word runs from the host, k_scatter into the plane layout)."""
    p = lambda x: os.path.join(c5_dir, x)
    _run([_bin("chainNet"), p("in.chain"), p("t.sizes"), p("q.sizes"), p("sp.t.net"),
          p("sp.q.net"), "-rescore", f"-tNibDir={p('t.2bit')}", f"-qNibDir={p('q.2bit')}",
          "-linearGap=loose"], env={"GAC_NET_SPARSE": "1"})
    _same(p("sp.t.net"), c5_ref_nets[0])
    _same(p("sp.q.net"), c5_ref_nets[1])


@pytest.mark.timeout(900)
@pytest.mark.parametrize("nranks,env", [(2, {}), (3, {}), (2, {"GAC_NET_SPARSE": "1"})])
def test_c5_shaped_chainnet_rescore_ranks(c5_dir, c5_ref_nets, nranks, env):
    """The multi-GPU mode (-nranks=N -rank=R, one process per rank): each
    rank nets and rescores its share of the chromosome sides, rank 0
    assembles both nets -- identical to the reference's single run.  (All
    ranks on device 0 here: the box has one GPU.)"""
    p = lambda x: os.path.join(c5_dir, x)
    tag = f"mr{nranks}{'s' if env else ''}"
    procs = [subprocess.Popen(
        [_bin("chainNet"), p("in.chain"), p("t.sizes"), p("q.sizes"), p(f"{tag}.t.net"),
         p(f"{tag}.q.net"), "-rescore", f"-tNibDir={p('t.2bit')}", f"-qNibDir={p('q.2bit')}",
         "-linearGap=loose", f"-nranks={nranks}", f"-rank={r}", "-gpu=0"],
        stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
        env=dict(os.environ, GAC_RANK_TOKEN=tag, **env)) for r in range(nranks)]
    for r, pr in enumerate(procs):
        _, err = pr.communicate(timeout=600)
        assert pr.returncode == 0, (r, err[-2000:])
    _same(p(f"{tag}.t.net"), c5_ref_nets[0])
    _same(p(f"{tag}.q.net"), c5_ref_nets[1])
    assert not [f for f in os.listdir(c5_dir) if ".gacsize" in f or ".gacdone" in f
                or (".gacpart" in f and tag in f)]


# ---------------------------------------------------------------- C2
@pytest.mark.timeout(900)
def test_c2_chainnet_rescore(tmp_path):
    from genomealignmenttools_amd import synth
    tg, qg, ca = synth.c2_case(seed=42, n_chains=200_000)
    _write_case(str(tmp_path), tg, qg, ca)
    del tg, qg, ca
    _rescore_pair(str(tmp_path), "c2")


# ---------------------------------------------------------------- C3
@pytest.mark.timeout(900)
def test_c3_chaincleaner(tmp_path):
    """Config C3 at hg38.mm10.chr1 scale: the C2 chain set plus 1000 planted
    chain-breaking-alignment loci (synth.c3_case), header scores from
    bin/scoreChain (byte-identical to the reference's), sorted and numbered;
    the net is the reference pipeline's: oracle/_ref/chainNet -minScore=0 |
    NetFilterNonNested -minScore1 3000 (the product's C build of the perl
    filter, byte-identical to /root/reference/src/NetFilterNonNested.perl on
    this very net in the build container and on the typed goldens of
    tests/test_host.py).  bin/chainCleaner -net= and oracle/_ref/chainCleaner
    -net= must write identical chains and removedSuspects beds, and the bed
    must be non-empty."""
    from genomealignmenttools_amd import chainfile, synth
    d = str(tmp_path)
    p = lambda x: os.path.join(d, x)
    tg, qg, ca = synth.c3_case(seed=42, n_chains=200_000, n_loci=1000)
    synth.write_2bit(tg, p("t.2bit"))
    synth.write_2bit(qg, p("q.2bit"))
    synth.write_sizes(tg.sizes, p("t.sizes"))
    synth.write_sizes(qg.sizes, p("q.sizes"))
    chainfile.write_chains_fast(ca, p("unscored.chain"))
    del tg, qg, ca
    _run([_bin("scoreChain"), p("unscored.chain"), p("t.2bit"), p("q.2bit"), p("sc.chain"),
          "-linearGap=loose"])
    sc = chainfile.read_chains(p("sc.chain"))
    sc = sc.subset(np.argsort(-sc.score, kind="stable"))
    sc.id = np.arange(1, sc.n + 1, dtype=np.int64)
    chainfile.write_chains_fast(sc, p("in.chain"))
    del sc
    net = _run([_ref("chainNet"), "-minScore=0", p("in.chain"), p("t.sizes"), p("q.sizes"),
                "stdout", "/dev/null"])
    filt = subprocess.run([_bin("NetFilterNonNested.perl"), "/dev/stdin", "-minScore1", "3000"],
                          input=net.stdout, capture_output=True, text=True, timeout=600)
    assert filt.returncode == 0, filt.stderr[-2000:]
    with open(p("in.net"), "w") as f:
        f.write(filt.stdout)
    del net, filt
    opts = [f"-net={p('in.net')}", "-linearGap=loose"]
    _run([_bin("chainCleaner"), p("in.chain"), p("t.2bit"), p("q.2bit"), p("ours.chain"),
          p("ours.bed")] + opts)
    ref_env = {"PATH": os.path.dirname(_ref("chainSort")) + os.pathsep + os.environ["PATH"]}
    _run([_ref("chainCleaner"), p("in.chain"), p("t.2bit"), p("q.2bit"), p("ref.chain"),
          p("ref.bed")] + opts, env=ref_env)
    _same(p("ours.chain"), p("ref.chain"))
    _same(p("ours.bed"), p("ref.bed"))
    with open(p("ref.bed")) as f:
        removed = sum(1 for _ in f)
    assert removed > 1000, removed


# ---------------------------------------------------------------- C4-shaped
@pytest.mark.timeout(900)
def test_c4_shaped_axtchain(tmp_path):
    from genomealignmenttools_amd import synth
    tg, qg, pairs, b = synth.psl_c4(7, 1_200_000, n_t=24, n_q=21, tsize=12_000_000,
                                    qsize=10_000_000)
    assert len(pairs) == 24 * 21 * 2 and len(b["t"]) > 1_000_000
    d = str(tmp_path)
    synth.write_2bit(tg, os.path.join(d, "t.2bit"))
    synth.write_2bit(qg, os.path.join(d, "q.2bit"))
    synth.write_psl_c4(tg, qg, pairs, b, os.path.join(d, "in.psl"), 7)
    del tg, qg, b
    args = ["-linearGap=loose", "-psl", "in.psl", "t.2bit", "q.2bit"]
    _run([_bin("axtChain")] + args + ["ours.chain"], cwd=d)
    _run([_ref("axtChain")] + args + ["ref.chain"], cwd=d)
    _same(os.path.join(d, "ours.chain"), os.path.join(d, "ref.chain"))
    # the kd-tree DP and the crossovers on the device (rows A13/A14)
    env = dict(os.environ, GAC_AXT_DP="gpu")
    r = subprocess.run([_bin("axtChain")] + args + ["gpu.chain"], cwd=d, env=env,
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr
    _same(os.path.join(d, "gpu.chain"), os.path.join(d, "ref.chain"))


@pytest.mark.timeout(1200)
def test_c4_shaped_axtchain_5m_blocks(tmp_path):
    """The C4 shape at 5 M PSL blocks (a tenth of SURVEY §8(d)'s 50 M; the
    reference takes about a minute here), the product's default -- the
    hybrid DP: the smaller pairs' kd-tree DP on the device (k_dp_fast), the
    others on host threads -- and the device DP alone (GAC_AXT_DP=gpu), byte
    for byte against the reference run in the same test."""
    from genomealignmenttools_amd import synth
    tg, qg, pairs, b = synth.psl_c4(7, 5_000_000, n_t=24, n_q=21, tsize=12_000_000,
                                    qsize=10_000_000)
    assert len(b["t"]) > 4_900_000
    d = str(tmp_path)
    synth.write_2bit(tg, os.path.join(d, "t.2bit"))
    synth.write_2bit(qg, os.path.join(d, "q.2bit"))
    synth.write_psl_c4(tg, qg, pairs, b, os.path.join(d, "in.psl"), 7)
    del tg, qg, b
    args = ["-linearGap=loose", "-psl", "in.psl", "t.2bit", "q.2bit"]
    r = _run([_bin("axtChain")] + args + ["ours.chain"], cwd=d, env={"GAC_TIMING": "1"})
    m = re.search(r"hybrid DP: (\d+) of (\d+) pairs \((\d+) of (\d+) blocks", r.stderr)
    assert m and int(m.group(1)) > 0 and int(m.group(3)) > 100_000, r.stderr[-3000:]
    _run([_bin("axtChain")] + args + ["dev.chain"], cwd=d, env={"GAC_AXT_DP": "gpu"})
    _run([_ref("axtChain")] + args + ["ref.chain"], cwd=d, timeout=900)
    _same(os.path.join(d, "ours.chain"), os.path.join(d, "ref.chain"))
    _same(os.path.join(d, "dev.chain"), os.path.join(d, "ref.chain"))


@pytest.mark.timeout(900)
def test_device_dp_fallbacks(tmp_path):
    """k_dp_spec's and k_dp_fast's two ways back to the reference walk, on the device: the
    anomaly check (an overlapping candidate whose crossover beats its bound,
    chainConnect.c:61-105) on a C4-shaped set dense with overlaps, and the
    overlap lists' cap (GAC_DP_OVCAP=0: every leaf with an overlapping
    candidate gets a -1 entry) -- both against the reference's chains, with
    the kernel's own count of fallbacks (GAC_DP_PROF) asserted non-zero."""
    synth = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                         "genomealignmenttools_amd", "libexec", "gac_synth")
    d = str(tmp_path)
    subprocess.run([synth, "c4", d, "-blocks=200000", "-nt=2", "-nq=2", "-tsize=3000000",
                    "-qsize=2500000", "-threads=4"], check=True, timeout=300, capture_output=True)
    args = ["-linearGap=loose", "-psl", "in.psl", "t.2bit", "q.2bit"]
    _run([_ref("axtChain")] + args + ["ref.chain"], cwd=d, timeout=600)
    counts = []
    # k_dp_spec (16 waves per pair, the default) and k_dp_fast (one wave)
    for waves in ("16", "1"):
        for cap in ("", "0"):
            out = "dev%s_%s.chain" % (cap, waves)
            r = _run([_bin("axtChain")] + args + [out], cwd=d,
                     env={"GAC_AXT_DP": "gpu", "GAC_DP_PROF": "1", "GAC_DP_OVCAP": cap,
                          "GAC_DP_WAVES": waves})
            m = re.search(r"(k_dp_(?:fast|spec)) .*?(\d+) leaves, (\d+) fallbacks", r.stderr)
            assert m and m.group(1) == ("k_dp_spec" if waves == "16" else "k_dp_fast"), r.stderr[-2000:]
            counts.append(int(m.group(3)))
            _same(os.path.join(d, out), os.path.join(d, "ref.chain"))
    assert counts[0] > 0 and counts[1] > counts[0], counts
    assert counts[2:] == counts[:2], counts


# ---------------------------------------------------------------- edge cases
def _synth(seed):
    return os.path.join(GOLDEN, f"synth{seed}")


@pytest.mark.parametrize("tool", ["scoreChain", "chainNet"])
def test_linear_gap_file(tool, tmp_path):
    """-linearGap=<file> (gapCalcRead, kent/src/lib/gapCalc.c:146-222) on the
    device gap path, against the reference with the same file."""
    d = _synth(11)
    p = lambda x: os.path.join(d, x)
    gap = "-linearGap=" + os.path.join(GOLDEN, "linearGap.txt")
    if tool == "scoreChain":
        for flag in ([], ["-returnOnlyScore"]):
            args = [p("in.chain"), p("t.2bit"), p("q.2bit")]
            _run([_bin("scoreChain")] + args + [tmp_path / "ours", gap] + flag)
            _run([_ref("scoreChain")] + args + [tmp_path / "ref", gap] + flag)
            _same(tmp_path / "ours", tmp_path / "ref")
    else:
        for f in ["in.chain", "t.2bit", "q.2bit", "t.sizes", "q.sizes"]:
            os.symlink(p(f), tmp_path / f)
        _rescore_pair(str(tmp_path), "lg", [gap])


def test_zero_size_end_blocks(tmp_path):
    """Chains whose first/last block has size 0: a full-chain query is
    chainFastSubsetOnT's easy case (kent/src/lib/chain.c:499-505), so those
    blocks and their gaps count in scoreChain's global and local scores."""
    from genomealignmenttools_amd import chainfile, synth
    d = _synth(12)
    p = lambda x: os.path.join(d, x)
    ca = synth.zero_end_blocks(chainfile.read_chains(p("in.chain")))
    chainfile.write_chains(ca, str(tmp_path / "in.chain"))
    for flag in (["-returnOnlyScoreAndCoords"], ["-forceLocalScore"], []):
        args = [tmp_path / "in.chain", p("t.2bit"), p("q.2bit")]
        _run([_bin("scoreChain")] + args + [tmp_path / "ours", "-linearGap=loose"] + flag)
        _run([_ref("scoreChain")] + args + [tmp_path / "ref", "-linearGap=loose"] + flag)
        _same(tmp_path / "ours", tmp_path / "ref")
    for f in ["t.2bit", "q.2bit", "t.sizes", "q.sizes"]:
        os.symlink(p(f), tmp_path / f)
    _rescore_pair(str(tmp_path), "z")


def test_chainnet_rescore_missing_sequence(tmp_path):
    """A chain on sequences listed in the .sizes files but absent from both
    .2bit files, which owns no rescored (partial) fill: the reference never
    looks its sequences up, so the run must succeed -- through the
    subset-upload branch of bin/chainNet -- with identical nets."""
    from genomealignmenttools_amd import chainfile, synth
    d = _synth(11)
    p = lambda x: os.path.join(d, x)
    ca = chainfile.read_chains(p("in.chain"))
    # one extra chain alone on new sequences chrTX / chrQX, lowest score
    lo = float(ca.score.min()) - 1
    from genomealignmenttools_amd.chainfile import ChainArrays
    extra = ChainArrays(score=np.array([max(lo, 1.0)]), tname=["chrTX"],
                        tsize=np.array([50_000], np.int32), tstart=np.array([100], np.int32),
                        tend=np.array([400], np.int32), qname=["chrQX"],
                        qsize=np.array([40_000], np.int32), qstrand=np.array([0], np.uint8),
                        qstart=np.array([200], np.int32), qend=np.array([520], np.int32),
                        id=np.array([ca.id.max() + 1], np.int64),
                        blk_off=np.array([0, 2], np.int64), blk_t=np.array([100, 300], np.int32),
                        blk_q=np.array([200, 420], np.int32), blk_size=np.array([100, 100], np.int32))
    both = synth.concat_chains([ca, extra])
    both = both.subset(np.argsort(-both.score, kind="stable"))
    chainfile.write_chains(both, str(tmp_path / "in.chain"))
    for side, new, size in (("t", "chrTX", 50_000), ("q", "chrQX", 40_000)):
        sizes = synth.read_sizes(p(f"{side}.sizes"))
        sizes[new] = size
        synth.write_sizes(sizes, str(tmp_path / f"{side}.sizes"))
        os.symlink(p(f"{side}.2bit"), tmp_path / f"{side}.2bit")
    _rescore_pair(str(tmp_path), "miss")


def test_chainnet_rescore_no_partial_fills(tmp_path):
    """-rescore where every printed fill covers its whole chain: nothing is
    rescored, the genomes are never read."""
    from genomealignmenttools_amd import chainfile, synth
    d = _synth(12)
    p = lambda x: os.path.join(d, x)
    ca = chainfile.read_chains(p("in.chain"))
    chainfile.write_chains(ca.subset(np.array([0])), str(tmp_path / "in.chain"))
    for f in ["t.2bit", "q.2bit", "t.sizes", "q.sizes"]:
        os.symlink(p(f), tmp_path / f)
    _rescore_pair(str(tmp_path), "one")


def test_chainnet_rescore_failures_exit_cleanly(tmp_path):
    """Failures while the device/upload helper threads are live end the
    process with errAbort's status 255 (no crash, no hang): a corrupt .2bit
    (the bring-up fails while the pre-upload helper waits for it) and an
    output on a full device (write error after the device close started)."""
    d = _synth(11)
    p = lambda x: os.path.join(d, x)
    with open(p("t.2bit"), "rb") as f:
        head = f.read(64)
    bad = tmp_path / "bad.2bit"
    bad.write_bytes(head)  # signature + a truncated index
    args = [p("in.chain"), p("t.sizes"), p("q.sizes")]
    r = _run([_bin("chainNet")] + args + [tmp_path / "t.net", tmp_path / "q.net", "-rescore",
                                          f"-tNibDir={bad}", f"-qNibDir={p('q.2bit')}",
                                          "-linearGap=loose"], rc=255, timeout=300)
    assert r.stderr.strip()
    if os.path.exists("/dev/full"):
        _run([_bin("chainNet")] + args + ["/dev/full", tmp_path / "q.net", "-rescore",
                                          f"-tNibDir={p('t.2bit')}", f"-qNibDir={p('q.2bit')}",
                                          "-linearGap=loose"], rc=255, timeout=300)


# ---------------------------------------------------------------- full scale
def _golden_full(which):
    with open(os.path.join(GOLDEN, "fullscale", f"{which}.json")) as f:
        return json.load(f)


def _sha(*paths):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    got = bench.sha256_files(list(paths))
    return [got[p] for p in paths]


@pytest.mark.timeout(900)
def test_c5_fullscale_vs_reference_sha(tmp_path):
    """C5 at the bench's full size (5 M chains, 116 M blocks, all 455 x 66
    sequences): bin/chainNet -rescore nets -- one process, and eight ranks
    (-nranks=8, the 8-GPU split) -- and bin/scoreChain's chains have the
    sha256 of the reference's outputs on the same input
    (tests/golden/fullscale/c5.json; the reference takes ~45 min for the
    nets, so its outputs are pinned by hash)."""
    from genomealignmenttools_amd._lib import PKG_DIR
    g = _golden_full("c5")
    d = str(tmp_path)
    p = lambda x: os.path.join(d, x)
    _run([os.path.join(PKG_DIR, "libexec", "gac_synth"), "c5", d, "-seed=1234", "-chains=5000000",
          f"-sizesDir={os.path.join(PKG_DIR, 'data')}", "-threads=16"])
    _run([_bin("chainNet"), p("in.chain"), p("t.sizes"), p("q.sizes"), p("o.t.net"), p("o.q.net"),
          "-rescore", f"-tNibDir={p('t.2bit')}", f"-qNibDir={p('q.2bit')}", "-linearGap=loose"])
    _run([_bin("scoreChain"), p("in.chain"), p("t.2bit"), p("q.2bit"), p("o.sc.chain"),
          "-linearGap=loose"])
    # the 8-GPU split of the headline (bench.py --gpus 8): chainNet -nranks=8,
    # every rank here on device 0 with 2 host threads
    procs = [subprocess.Popen([_bin("chainNet"), p("in.chain"), p("t.sizes"), p("q.sizes"),
                               p("r8.t.net"), p("r8.q.net"), "-rescore", f"-tNibDir={p('t.2bit')}",
                               f"-qNibDir={p('q.2bit')}", "-linearGap=loose", "-nranks=8",
                               f"-rank={r}", "-gpu=0"],
                              stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                              env=dict(os.environ, GAC_RANK_TOKEN="c5r8", GAC_THREADS="2"))
             for r in range(8)]
    for r, pr in enumerate(procs):
        _, err = pr.communicate(timeout=600)
        assert pr.returncode == 0, (r, err[-2000:])
    i, t, q, sc, t8, q8 = _sha(p("in.chain"), p("o.t.net"), p("o.q.net"), p("o.sc.chain"),
                               p("r8.t.net"), p("r8.q.net"))
    assert i == g["in_chain_sha256"], "generated input differs from the golden run's"
    assert t == g["chainnet_rescore"]["t_net_sha256"]
    assert q == g["chainnet_rescore"]["q_net_sha256"]
    assert sc == g["scorechain"]["chain_sha256"]
    assert t8 == g["chainnet_rescore"]["t_net_sha256"]
    assert q8 == g["chainnet_rescore"]["q_net_sha256"]
    assert not [f for f in os.listdir(d) if ".gacpart" in f or ".gacsize" in f or ".gacdone" in f]


@pytest.mark.timeout(900)
def test_c4_fullscale_axtchain_vs_reference_sha(tmp_path):
    """C4 at the SURVEY size (gac_synth c4: 50 M PSL blocks over 24 x 21 pairs
    x 2 strands, largest pair 11.5 M blocks): bin/axtChain, one process and
    -nranks=3 (seqPairs dealt out, rank 0 merges; all ranks on device 0
    here), has the sha256 of the reference axtChain's output
    (tests/golden/fullscale/c4.json: ~21 min for the reference)."""
    from genomealignmenttools_amd._lib import PKG_DIR
    g = _golden_full("c4")
    d = str(tmp_path)
    _run([os.path.join(PKG_DIR, "libexec", "gac_synth"), "c4", d, "-seed=7", "-blocks=50000000",
          "-threads=16"])
    args = ["-linearGap=loose", "-verbose=0", "-psl", "in.psl", "t.2bit", "q.2bit"]
    r = _run([_bin("axtChain")] + args + ["one.chain"], cwd=d, env={"GAC_TIMING": "1"})
    # the default hybrid DP put a share of the pairs' leaves on the device
    m = re.search(r"hybrid DP: (\d+) of (\d+) pairs \((\d+) of (\d+) blocks", r.stderr)
    assert m and int(m.group(3)) > 1_000_000, r.stderr[-3000:]
    procs = [subprocess.Popen([_bin("axtChain")] + args + ["r3.chain", "-nranks=3", f"-rank={r}",
                                                           "-gpu=0"], cwd=d,
                              stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                              env=dict(os.environ, GAC_RANK_TOKEN="c4r3", GAC_THREADS="6"))
             for r in range(3)]
    for r, pr in enumerate(procs):
        _, err = pr.communicate(timeout=600)
        assert pr.returncode == 0, (r, err[-2000:])
    i, one, r3 = _sha(os.path.join(d, "in.psl"), os.path.join(d, "one.chain"),
                      os.path.join(d, "r3.chain"))
    assert i == g["in_psl_sha256"], "generated input differs from the golden run's"
    assert one == g["axtchain"]["chain_sha256"]
    assert r3 == g["axtchain"]["chain_sha256"]
