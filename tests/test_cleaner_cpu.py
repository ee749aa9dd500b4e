"""chainCleaner's host logic on CPU: oracle/_build/chainCleaner_cpu is the
real tool on the CPU stand-in of the device ABI (oracle/cpu_gac_stub.c, TEST
INFRASTRUCTURE: plain reference arithmetic for the scores).  Every golden
case (the reference's outputs, tests/golden/cleaner) with

- GAC_CLEANER_CHECK_KEYS=1: each sub-chain key's version decided from the
  blocks removed so far is checked against the rule it replaces (the counts
  of the current and the original selections, chainSubsetOnT on both);
- the speculative keys and per-list batches on (default) and off
  (GAC_CLEANER_SPEC=0): scoring order must not change a decision.
"""
import filecmp
import json
import os
import subprocess

import pytest

from conftest import GOLDEN

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TOOL = os.path.join(ROOT, "oracle", "_build", "chainCleaner_cpu")


@pytest.fixture(scope="module")
def tool():
    import fcntl
    os.makedirs(os.path.join(ROOT, "oracle", "_build"), exist_ok=True)
    with open(os.path.join(ROOT, "oracle", "_build", ".cpu-chaincleaner.lock"), "w") as lk:
        fcntl.flock(lk, fcntl.LOCK_EX)
        r = subprocess.run(["make", "-s", "cpu-chaincleaner"], cwd=ROOT, capture_output=True,
                           text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    return TOOL


def _cases():
    with open(os.path.join(GOLDEN, "cleaner", "cases.json")) as f:
        return json.load(f)


@pytest.mark.parametrize("spec", ["1", "0"])
@pytest.mark.parametrize("case", ["default", "pairs", "lowfold", "filters", "sdata", "debug"])
def test_cleaner_cpu_vs_golden(tool, case, spec, tmp_path):
    d = os.path.join(GOLDEN, "cleaner")
    cases = _cases()
    opts = cases["cases"][case]
    p = lambda x: os.path.join(d, x)
    cmd = [tool, p("in.chain"), p("t.2bit"), p("q.2bit"), "out.chain", "out.bed", f"-net={p('in.net')}"]
    env = dict(os.environ, GAC_CLEANER_CHECK_KEYS="1", GAC_CLEANER_SPEC=spec, GAC_THREADS="2")
    r = subprocess.run(cmd + opts, capture_output=True, text=True, timeout=600, cwd=tmp_path, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    files = ["out.chain", "out.bed"]
    for o in opts:
        if o.startswith("-newChainIDDict=") or o.startswith("-suspectDataFile="):
            files.append(o.split("=", 1)[1])
    if "-debug" in opts:
        files += cases["debug_files"]
    for f in files:
        assert filecmp.cmp(tmp_path / f, os.path.join(d, case, f), shallow=False), (case, f)
