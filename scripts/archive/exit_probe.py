#!/usr/bin/env python3
"""Probe (measurement only): where process exit time goes.  Runs each
command a few times and reports, from the "[stage-clock] exit" anchor the
program prints just before _exit, the time until the parent's wait returns
(process teardown), plus the whole wall time.  Usage:
  exit_probe.py REPS -- cmd1 args ;; cmd2 args ;; ..."""
import subprocess
import sys
import time


def run(cmd):
    t0 = time.time()
    r = subprocess.run(cmd, capture_output=True, text=True)
    t1 = time.time()
    ex = None
    for line in r.stderr.splitlines():
        if line.startswith("[stage-clock] exit"):
            ex = float(line.split()[2])
    return r.returncode, t1 - t0, (t1 - ex) if ex else None, r.stderr


def main():
    reps = int(sys.argv[1])
    cmds, cur = [], []
    for a in sys.argv[3:]:
        if a == ";;":
            cmds.append(cur)
            cur = []
        else:
            cur.append(a)
    if cur:
        cmds.append(cur)
    for cmd in cmds:
        res = [run(cmd) for _ in range(reps)]
        rcs = {r[0] for r in res}
        walls = " ".join(f"{r[1]:.3f}" for r in res)
        exits = " ".join(f"{r[2]:.3f}" if r[2] is not None else "-" for r in res)
        print(f"{' '.join(cmd)[-120:]}\n  rc={rcs} wall {walls}  exit->wait {exits}", flush=True)
        if rcs != {0}:
            print(res[-1][3][-1500:], flush=True)


if __name__ == "__main__":
    main()
