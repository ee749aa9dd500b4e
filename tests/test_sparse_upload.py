"""chainNet -rescore's sparse genome upload, checked on CPU.

The tool uploads only the 32-base words under its chains' blocks
(gt_runs_build, tools/lib/gac_tool.c).  oracle/_build/chainNet_cpu is the
real tool linked against the CPU stand-in of the device ABI
(oracle/cpu_gac_stub.c), which poisons every word outside the runs: a run set
that misses a word the fill rescoring reads changes a score.  The nets must
equal the whole-genome run (the default; GAC_NET_SPARSE=1 turns the sparse
upload on) and, when it is built, the
reference chainNet (oracle/_ref).  TEST INFRASTRUCTURE only.
"""
import filecmp
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TOOL = os.path.join(ROOT, "oracle", "_build", "chainNet_cpu")


@pytest.fixture(scope="module")
def tool():
    # one build at a time: pytest-xdist workers may reach this together
    import fcntl
    os.makedirs(os.path.join(ROOT, "oracle", "_build"), exist_ok=True)
    with open(os.path.join(ROOT, "oracle", "_build", ".cpu-chainnet.lock"), "w") as lk:
        fcntl.flock(lk, fcntl.LOCK_EX)
        r = subprocess.run(["make", "-s", "cpu-chainnet"], cwd=ROOT, capture_output=True,
                           text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    return TOOL


def _case(d, kind, seed):
    from genomealignmenttools_amd import chainfile, synth
    if kind == "small":
        tg, qg, ca = synth.small_case(seed=seed, n_chains=400)
    elif kind == "zero_end":
        tg, qg, ca = synth.small_case(seed=seed, n_chains=300)
        ca = synth.zero_end_blocks(ca, every=2)
    else:  # C5-shaped: every hg38/mm10 name, both strands, shrunk sequences
        tg, qg, ca = synth.c5_case(seed=seed, n_chains=6000, scale=0.002, min_size=20_000)
    synth.write_2bit(tg, os.path.join(d, "t.2bit"))
    synth.write_2bit(qg, os.path.join(d, "q.2bit"))
    synth.write_sizes(tg.sizes, os.path.join(d, "t.sizes"))
    synth.write_sizes(qg.sizes, os.path.join(d, "q.sizes"))
    chainfile.write_chains(ca, os.path.join(d, "in.chain"))


def _net(exe, d, tag, env=None, extra=()):
    p = lambda x: os.path.join(d, x)
    cmd = [exe, p("in.chain"), p("t.sizes"), p("q.sizes"), p(f"{tag}.t.net"), p(f"{tag}.q.net"),
           "-rescore", f"-tNibDir={p('t.2bit')}", f"-qNibDir={p('q.2bit')}",
           "-linearGap=loose"] + list(extra)
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, **(env or {})))
    assert r.returncode == 0, r.stderr[-2000:]
    return p(f"{tag}.t.net"), p(f"{tag}.q.net")


@pytest.mark.parametrize("kind,seed", [("small", 3), ("small", 11), ("zero_end", 5),
                                       ("c5", 21)])
def test_sparse_runs_cover_rescoring(tool, tmp_path, kind, seed):
    d = str(tmp_path)
    _case(d, kind, seed)
    sparse = _net(tool, d, "sparse", env={"GAC_NET_SPARSE": "1"})
    whole = _net(tool, d, "whole", env={"GAC_NET_SPARSE": "0"})
    for a, b in zip(sparse, whole):
        assert filecmp.cmp(a, b, shallow=False), f"{a} differs from {b}"
    # the poisoning is live: some fill was rescored (a partial fill's score
    # line differs from its chain's score in a rescored net)
    assert os.path.getsize(sparse[0]) > 0
    from oracle.oracle import ref_tool
    ref = ref_tool("chainNet")
    if os.path.exists(ref):
        refd = _net(ref, d, "ref")
        for a, b in zip(sparse, refd):
            assert filecmp.cmp(a, b, shallow=False), f"{a} differs from {b}"


def test_poisoned_words_change_scores(tool, tmp_path):
    """Guard for the check itself: with every word poisoned (runs built from
    an empty chain set would be), rescored partial fills change."""
    d = str(tmp_path)
    _case(d, "small", 3)
    whole = _net(tool, d, "whole", env={"GAC_NET_SPARSE": "0"})
    poisoned = _net(tool, d, "poison", env={"GAC_NET_SPARSE": "1", "GAC_STUB_POISON_ALL": "1"})
    assert not filecmp.cmp(whole[0], poisoned[0], shallow=False)
