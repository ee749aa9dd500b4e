"""GPU end-to-end parity of the drop-in tools against the reference's own
outputs (tests/golden, generated with the tools compiled from
/root/reference): byte-identical files."""
import filecmp
import json
import os
import subprocess

import numpy as np
import pytest

from conftest import BLASTZ, GOLDEN

pytestmark = pytest.mark.gpu


def _bin(name):
    from genomealignmenttools_amd._lib import BIN_DIR
    return os.path.join(BIN_DIR, name)


def _run(cmd):
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr
    return r


@pytest.mark.parametrize("case", ["newStyleLastz", "oldStyleBlastz"])
@pytest.mark.parametrize("gap", ["loose", "medium"])
@pytest.mark.parametrize("mode,flag", [("score", "-returnOnlyScore"),
                                       ("coords", "-returnOnlyScoreAndCoords"),
                                       ("chain", None), ("local", "-forceLocalScore")])
def test_scorechain_chrM(case, gap, mode, flag, tmp_path):
    d = os.path.join(GOLDEN, "chrM")
    out = tmp_path / "out"
    cmd = [_bin("scoreChain"), os.path.join(d, f"{case}.chain"), os.path.join(d, "hg19.chrM.2bit"),
           os.path.join(d, "susScr3.chrM.2bit"), str(out), f"-linearGap={gap}",
           f"-scoreScheme={os.path.join(d, case + '.Q.txt')}"]
    if flag:
        cmd.append(flag)
    _run(cmd)
    assert filecmp.cmp(out, os.path.join(d, f"{case}.{gap}.{mode}.out"), shallow=False)


@pytest.mark.parametrize("seed", [11, 12])
def test_scorechain_synth(seed, tmp_path):
    d = os.path.join(GOLDEN, f"synth{seed}")
    p = lambda x: os.path.join(d, x)
    _run([_bin("scoreChain"), p("in.chain"), p("t.2bit"), p("q.2bit"), str(tmp_path / "a"),
          "-linearGap=loose", "-returnOnlyScoreAndCoords"])
    assert filecmp.cmp(tmp_path / "a", p("score.out"), shallow=False)
    _run([_bin("scoreChain"), p("in.chain"), p("t.2bit"), p("q.2bit"), str(tmp_path / "b"),
          "-linearGap=medium", "-doLocalScore"])
    assert filecmp.cmp(tmp_path / "b", p("rescored.chain"), shallow=False)


@pytest.mark.parametrize("seed", [11, 12])
def test_chainnet_rescore_synth(seed, tmp_path):
    d = os.path.join(GOLDEN, f"synth{seed}")
    p = lambda x: os.path.join(d, x)
    _run([_bin("chainNet"), p("in.chain"), p("t.sizes"), p("q.sizes"), str(tmp_path / "t.net"),
          str(tmp_path / "q.net"), "-rescore", f"-tNibDir={p('t.2bit')}",
          f"-qNibDir={p('q.2bit')}", "-linearGap=loose"])
    assert filecmp.cmp(tmp_path / "t.net", p("rescore.t.net"), shallow=False)
    assert filecmp.cmp(tmp_path / "q.net", p("rescore.q.net"), shallow=False)


@pytest.mark.parametrize("mode", ["gz", "stdin"])
def test_stream_inputs_and_stdout(mode, tmp_path):
    """kent file-name conventions on the GPU tools: a .gz chain file (read
    through gzip, lineFileOpen) or `stdin` as the input, `stdout` as
    scoreChain's output; same bytes as the reference's goldens."""
    import gzip
    import shutil
    d = os.path.join(GOLDEN, "synth11")
    p = lambda x: os.path.join(d, x)
    src = p("in.chain")
    if mode == "gz":
        with open(src, "rb") as f, gzip.open(tmp_path / "in.chain.gz", "wb") as g:
            shutil.copyfileobj(f, g)
        src = str(tmp_path / "in.chain.gz")

    def run(cmd):
        with open(p("in.chain"), "rb") as fin:
            r = subprocess.run([c if c != "IN" else ("stdin" if mode == "stdin" else src)
                                for c in cmd], stdin=fin if mode == "stdin" else None,
                               capture_output=True, timeout=600)
        assert r.returncode == 0, r.stderr[-2000:]
        return r.stdout

    out = run([_bin("scoreChain"), "IN", p("t.2bit"), p("q.2bit"), "stdout", "-linearGap=loose",
               "-returnOnlyScoreAndCoords"])
    assert out == open(p("score.out"), "rb").read()
    run([_bin("chainNet"), "IN", p("t.sizes"), p("q.sizes"), str(tmp_path / "t.net"),
         str(tmp_path / "q.net"), "-rescore", f"-tNibDir={p('t.2bit')}", f"-qNibDir={p('q.2bit')}",
         "-linearGap=loose"])
    assert filecmp.cmp(tmp_path / "t.net", p("rescore.t.net"), shallow=False)
    assert filecmp.cmp(tmp_path / "q.net", p("rescore.q.net"), shallow=False)


@pytest.mark.parametrize("seed", [11, 12])
@pytest.mark.parametrize("tag,opts", [("ms1", ["-minSpace=1", "-minScore=0"]),
                                      ("ms100", ["-minSpace=100", "-minFill=10"])])
def test_chainnet_rescore_options(seed, tag, opts, tmp_path):
    """-rescore with the medium gap table and space/fill/score thresholds
    (tests/golden/make_golden.py::net_variants, reference chainNet)."""
    d = os.path.join(GOLDEN, f"synth{seed}")
    p = lambda x: os.path.join(d, x)
    _run([_bin("chainNet"), p("in.chain"), p("t.sizes"), p("q.sizes"), str(tmp_path / "t.net"),
          str(tmp_path / "q.net"), "-rescore", f"-tNibDir={p('t.2bit')}",
          f"-qNibDir={p('q.2bit')}", "-linearGap=medium"] + opts)
    assert filecmp.cmp(tmp_path / "t.net", p(f"rescore_{tag}.t.net"), shallow=False)
    assert filecmp.cmp(tmp_path / "q.net", p(f"rescore_{tag}.q.net"), shallow=False)


@pytest.mark.parametrize("seed", [11, 12])
def test_api_subchains_vs_reference(seed):
    """The C ABI's batched sub-chain scores == reference chainSubsetOnT +
    chainCalcScore (+ scoreChain local loop) on 3000 random ranges."""
    from genomealignmenttools_amd.chainfile import read_chains
    from genomealignmenttools_amd.gachain import GAC_Q, GAC_T, Engine, GapCosts
    d = os.path.join(GOLDEN, f"synth{seed}")
    z = np.load(os.path.join(d, "subchain.npz"))
    ca = read_chains(os.path.join(d, "in.chain"))
    e = Engine(0)
    e.load_2bit(GAC_T, os.path.join(d, "t.2bit"))
    e.load_2bit(GAC_Q, os.path.join(d, "q.2bit"))
    e.set_scoring(np.asarray(BLASTZ, np.int32), GapCosts("loose"))
    cs = e.upload_chains(ca)
    g, l, a = e.score_ranges(cs, z["ranges"], want_local=True)
    assert np.array_equal(g, z["glob"]) and np.array_equal(l, z["loc"])
    assert np.array_equal(a, z["ali"])


def test_scorechain_c1_example(tmp_path):
    """Config C1: example/hg38.danRer10.chain with HoxD55.q against the seeded
    synthetic hg38 chr2 / danRer10 chr22 genomes (regenerated here)."""
    from genomealignmenttools_amd import synth
    d = os.path.join(GOLDEN, "c1")
    cfg = json.load(open(os.path.join(d, "seed.json")))
    s = cfg["seed"]
    tg = synth.random_genome(cfg["t"], s, n_frac=cfg["n_frac"], n_mean=cfg["n_mean"],
                             mask_frac=cfg["mask_frac"])
    qg = synth.random_genome(cfg["q"], s + 1, n_frac=cfg["n_frac"], n_mean=cfg["n_mean"],
                             mask_frac=cfg["mask_frac"])
    synth.write_2bit(tg, str(tmp_path / "t.2bit"))
    synth.write_2bit(qg, str(tmp_path / "q.2bit"))
    for mode, flag in [("score", "-returnOnlyScore"), ("chain", None)]:
        cmd = [_bin("scoreChain"), os.path.join(d, "hg38.danRer10.chain"), str(tmp_path / "t.2bit"),
               str(tmp_path / "q.2bit"), str(tmp_path / mode), "-linearGap=loose",
               "-scoreScheme=" + os.path.join(d, "HoxD55.q")]
        if flag:
            cmd.append(flag)
        _run(cmd)
        assert filecmp.cmp(tmp_path / mode, os.path.join(d, f"c1.{mode}.out"), shallow=False)


# ---------------------------------------------------------------- chainCleaner
def _cleaner_cases():
    with open(os.path.join(GOLDEN, "cleaner", "cases.json")) as f:
        return json.load(f)


def _cleaner_outputs(opts):
    files = ["out.chain", "out.bed"]
    for o in opts:
        if o.startswith("-newChainIDDict=") or o.startswith("-suspectDataFile="):
            files.append(o.split("=", 1)[1])
    if "-debug" in opts:
        files += _cleaner_cases()["debug_files"]
    return files


def _run_cleaner(case, tmp_path, net, env=None):
    d = os.path.join(GOLDEN, "cleaner")
    opts = _cleaner_cases()["cases"][case]
    p = lambda x: os.path.join(d, x)
    cmd = [_bin("chainCleaner"), p("in.chain"), p("t.2bit"), p("q.2bit"), "out.chain", "out.bed"]
    cmd += [f"-net={p('in.net')}"] if net else [f"-tSizes={p('t.sizes')}", f"-qSizes={p('q.sizes')}"]
    r = subprocess.run(cmd + opts, capture_output=True, text=True, timeout=600, cwd=tmp_path,
                       env=dict(os.environ, **(env or {})))
    assert r.returncode == 0, r.stderr
    for f in _cleaner_outputs(opts):
        assert filecmp.cmp(tmp_path / f, os.path.join(d, case, f), shallow=False), (case, f)


@pytest.mark.parametrize("case", ["default", "pairs", "lowfold", "filters", "sdata", "debug"])
def test_chaincleaner_net(case, tmp_path):
    """chainCleaner -net=in.net: every output byte-identical to the reference."""
    _run_cleaner(case, tmp_path, net=True)


@pytest.mark.parametrize("case", ["default", "pairs", "debug"])
def test_chaincleaner_net_launches(case, tmp_path):
    """The same with a k_small launch per on-demand batch (GAC_SMALL_SERVER=0)
    instead of the default resident small-batch server."""
    _run_cleaner(case, tmp_path, net=True, env={"GAC_SMALL_SERVER": "0"})


@pytest.mark.parametrize("case", ["default", "lowfold"])
def test_chaincleaner_nonet(case, tmp_path):
    """Without -net the tool nets in-process (chainNet -minScore=0 |
    NetFilterNonNested.perl -minScore1 3000); same outputs as the reference
    run on that pipeline's net."""
    _run_cleaner(case, tmp_path, net=False)


# ---------------------------------------------------------------- axtChain
@pytest.mark.parametrize("case", ["newStyleLastz", "oldStyleBlastz"])
def test_axtchain_kat(case, tmp_path):
    """The reference's own axtChain known-answer test
    (kent/src/hg/mouseStuff/axtChain/tests/makefile): -psl input, real chrM
    DNA, lastz matrices; byte-identical to tests/expected."""
    d = os.path.join(GOLDEN, "chrM")
    out = tmp_path / "out.chain"
    _run([_bin("axtChain"), "-psl", os.path.join(d, f"{case}.psl"), "-minScore=3000",
          "-linearGap=loose", os.path.join(d, "hg19.chrM.2bit"),
          f"-scoreScheme={os.path.join(d, case + '.Q.txt')}", os.path.join(d, "susScr3.chrM.2bit"),
          str(out)])
    assert filecmp.cmp(out, os.path.join(d, f"{case}.chain"), shallow=False)


def test_axtchain_kat_fasta(tmp_path):
    """-faQ/-faT: the same known answer with fasta genomes."""
    from oracle.oracle import read_2bit_text
    d = os.path.join(GOLDEN, "chrM")
    for name in ["hg19", "susScr3"]:
        seqs = read_2bit_text(os.path.join(d, f"{name}.chrM.2bit"))
        with open(tmp_path / f"{name}.fa", "w") as f:
            for k, v in seqs.items():
                f.write(f">{k}\n{v.decode()}\n")
    out = tmp_path / "out.chain"
    _run([_bin("axtChain"), "-psl", "-faQ", "-faT", os.path.join(d, "newStyleLastz.psl"),
          "-minScore=3000", "-linearGap=loose", str(tmp_path / "hg19.fa"),
          f"-scoreScheme={os.path.join(d, 'newStyleLastz.Q.txt')}", str(tmp_path / "susScr3.fa"),
          str(out)])
    assert filecmp.cmp(out, os.path.join(d, "newStyleLastz.chain"), shallow=False)


@pytest.mark.parametrize("seed", [5, 6])
@pytest.mark.parametrize("case", ["loose", "medium0", "hoxd", "axt"])
def test_axtchain_synth(seed, case, tmp_path):
    """Planted PSL/axt blocks with partial, exact and one-sided overlaps,
    noise, both strands: chains (and -details) byte-identical to the
    reference axtChain."""
    d = os.path.join(GOLDEN, "axtchain", f"s{seed}")
    with open(os.path.join(GOLDEN, "axtchain", "cases.json")) as f:
        opts = json.load(f)[case]
    inp = "in.psl" if "-psl" in opts else "in.axt.gz"
    opts = [o.replace("../../chrM", os.path.join(GOLDEN, "chrM")) for o in opts]
    r = subprocess.run([_bin("axtChain")] + opts + [os.path.join(d, inp), os.path.join(d, "t.2bit"),
                                                    os.path.join(d, "q.2bit"), "out.chain"],
                       capture_output=True, text=True, timeout=600, cwd=tmp_path)
    assert r.returncode == 0, r.stderr
    assert filecmp.cmp(tmp_path / "out.chain", os.path.join(d, f"{case}.chain"), shallow=False)
    for o in opts:
        if o.startswith("-details="):
            fn = o.split("=", 1)[1]
            assert filecmp.cmp(tmp_path / fn, os.path.join(d, fn), shallow=False)


@pytest.mark.parametrize("seed", [5, 6])
@pytest.mark.parametrize("case", ["loose", "medium0", "axt"])
def test_axtchain_synth_ranks(seed, case, tmp_path):
    """axtChain -nranks=2/3 (one process per rank, all on device 0 here):
    seqPairs dealt out by block count, rank 0 merges by (score, pair) --
    byte-identical to the reference's single run (the golden files)."""
    d = os.path.join(GOLDEN, "axtchain", f"s{seed}")
    with open(os.path.join(GOLDEN, "axtchain", "cases.json")) as f:
        opts = json.load(f)[case]
    inp = "in.psl" if "-psl" in opts else "in.axt.gz"
    args = opts + [os.path.join(d, inp), os.path.join(d, "t.2bit"), os.path.join(d, "q.2bit"),
                   "out.chain"]
    for n in (2, 3):
        env = dict(os.environ, GAC_RANK_TOKEN=f"s{seed}{case}{n}")
        procs = [subprocess.Popen([_bin("axtChain")] + args + [f"-nranks={n}", f"-rank={r}", "-gpu=0"],
                                  cwd=tmp_path, env=env, stdout=subprocess.PIPE,
                                  stderr=subprocess.PIPE, text=True) for r in range(n)]
        for r, pr in enumerate(procs):
            _, err = pr.communicate(timeout=300)
            assert pr.returncode == 0, (r, err[-2000:])
        assert filecmp.cmp(tmp_path / "out.chain", os.path.join(d, f"{case}.chain"), shallow=False)


@pytest.mark.parametrize("dp", ["host", "gpu"])
def test_axtchain_jobs_batch(dp, tmp_path):
    """axtChain -jobs=FILE: the two reference KATs and
    the 8 synthetic cases as one batch -- genomes switch between jobs, one
    device context -- every output identical to its golden file.  dp=gpu:
    the kd-tree DP and the chains' crossovers on the device (GAC_AXT_DP=gpu:
    k_dp, k_xover), rows A13/A14."""
    env = dict(os.environ, GAC_AXT_DP=dp)
    g = GOLDEN
    lines, expect = [], []
    for c in ["newStyleLastz", "oldStyleBlastz"]:
        out = tmp_path / f"kat_{c}.chain"
        lines.append(f"-psl {g}/chrM/{c}.psl -minScore=3000 -linearGap=loose {g}/chrM/hg19.chrM.2bit "
                     f"-scoreScheme={g}/chrM/{c}.Q.txt {g}/chrM/susScr3.chrM.2bit {out}")
        expect.append((out, os.path.join(g, "chrM", f"{c}.chain")))
    with open(os.path.join(g, "axtchain", "cases.json")) as f:
        cases = json.load(f)
    for seed in (5, 6):
        d = os.path.join(g, "axtchain", f"s{seed}")
        for case, opts in cases.items():
            opts = [o.replace("../../chrM", os.path.join(g, "chrM")) for o in opts]
            opts = [f"-details={tmp_path}/s{seed}.details" if o.startswith("-details=") else o
                    for o in opts]
            if any(o.startswith("-details=") for o in opts):
                expect.append((tmp_path / f"s{seed}.details", os.path.join(d, "hoxd.details")))
            inp = "in.psl" if "-psl" in opts else "in.axt.gz"
            out = tmp_path / f"s{seed}_{case}.chain"
            lines.append(" ".join(opts + [os.path.join(d, inp), os.path.join(d, "t.2bit"),
                                          os.path.join(d, "q.2bit"), str(out)]))
            expect.append((out, os.path.join(d, f"{case}.chain")))
    jobs = tmp_path / "jobs.txt"
    jobs.write_text("# one axtChain run per line\n\n" + "\n".join(lines) + "\n")
    r = subprocess.run([_bin("axtChain"), f"-jobs={jobs}"], capture_output=True, text=True,
                       timeout=600, cwd=tmp_path, env=env)
    assert r.returncode == 0, r.stderr
    for got, want in expect:
        assert filecmp.cmp(got, want, shallow=False), got
    # a failing job stops the batch with the reference's error and status
    bad = tmp_path / "bad.txt"
    bad.write_text(lines[0] + "\n" + f"-linearGap=loose {tmp_path}/missing.axt "
                   f"{g}/chrM/hg19.chrM.2bit {g}/chrM/susScr3.chrM.2bit {tmp_path}/x.chain\n")
    r = subprocess.run([_bin("axtChain"), f"-jobs={bad}"], capture_output=True, text=True,
                       timeout=600, cwd=tmp_path, env=env)
    assert r.returncode == 255 and "missing.axt" in r.stderr
