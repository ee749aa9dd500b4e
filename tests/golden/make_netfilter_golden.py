#!/usr/bin/env python3
"""Golden fixtures for the native NetFilterNonNested.perl drop-in: the
reference script (/root/reference/src/NetFilterNonNested.perl, run with the
system perl) on nets produced by the reference chainNet.

Run in the build container:  python tests/golden/make_netfilter_golden.py

tests/golden/netfilter/
  <net>.net           inputs: the reference chainNet's plain target nets of
                      synth11/synth12 and its -minScore=0 net of the cleaner
                      set (chainCleaner's own self-netting input)
  <net>.<case>.out    the perl script's output
  cases.json          option lists
"""
import json
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
PERL = "/root/reference/src/NetFilterNonNested.perl"
REF_BIN = os.path.join(REPO, "oracle", "_ref")
OUT = os.path.join(HERE, "netfilter")

CASES = {
    "s3000": ["-minScore1", "3000"],
    "two_sets": ["-minScore1", "10000", "-minSizeT1", "500", "-minSizeQ1", "500", "-minScore2",
                 "50000"],
    "eq": ["-minScore1=5000", "-minSizeQ1=200"],
    "batch": ["-minScore", "3000,20000,200000", "-minSizeT", "1000,0,0", "-minSizeQ", "1000,300,0"],
}


def main():
    os.makedirs(OUT, exist_ok=True)
    shutil.copy(os.path.join(HERE, "synth11", "plain.t.net"), os.path.join(OUT, "synth11.net"))
    shutil.copy(os.path.join(HERE, "synth12", "plain.q.net"), os.path.join(OUT, "synth12q.net"))
    c = os.path.join(HERE, "cleaner")
    net = subprocess.run([os.path.join(REF_BIN, "chainNet"), "-minScore=0", os.path.join(c, "in.chain"),
                          os.path.join(c, "t.sizes"), os.path.join(c, "q.sizes"), "stdout",
                          "/dev/null"], capture_output=True, text=True, check=True).stdout
    with open(os.path.join(OUT, "cleaner.net"), "w") as f:
        f.write(net)
    for name in ["synth11", "synth12q", "cleaner"]:
        for case, opts in CASES.items():
            r = subprocess.run(["perl", PERL, os.path.join(OUT, f"{name}.net")] + opts,
                               capture_output=True, text=True)
            assert r.returncode == 0, r.stderr
            with open(os.path.join(OUT, f"{name}.{case}.out"), "w") as f:
                f.write(r.stdout)
            print(name, case, r.stdout.count("fill"), "fills kept", file=sys.stderr)
    with open(os.path.join(OUT, "cases.json"), "w") as f:
        json.dump(CASES, f, indent=1)


if __name__ == "__main__":
    main()
