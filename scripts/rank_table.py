#!/usr/bin/env python3
"""DESIGN §6's per-rank tables from a solo-rank run (scripts/gpu_r05_ranks.sh:
every rank of chainNet / axtChain -nranks=N run alone with GAC_RANK_SOLO=1
and GAC_TIMING=1).  usage: rank_table.py DIR  -> markdown on stdout"""
import glob
import os
import re
import sys


def stages(text):
    out = {}
    for m in re.finditer(r"^\[stage\] (.+?)\s{2,}([0-9.]+) s", text, re.M):
        out[m.group(1).strip()] = float(m.group(2))
    return out


def main(d):
    rows = []
    for path in sorted(glob.glob(os.path.join(d, "c5_n*_r*.err")),
                       key=lambda p: tuple(int(x) for x in re.findall(r"\d+", os.path.basename(p))[1:3])):
        n, r = (int(x) for x in re.findall(r"_n(\d+)_r(\d+)", path)[0])
        t = open(path).read()
        wall = int(re.search(r"wall (\d+) ms", t).group(1))
        st = stages(t)
        side = re.search(r"sides: (\d+) target seqs \((\d+) bases\), (\d+) query seqs \((\d+) bases\); "
                         r"(\d+) chain headers, (\d+) blocks parsed; fills: (\d+) target, (\d+) query", t)
        parts = dict(re.findall(r"\] (target|query) net part: (\d+) bytes", t))
        rows.append((n, r, wall, st, side, parts))
    print("| N | rank | wall ms | target Mb | blocks parsed (M) | target fills (M) | read | netting | "
          "fill list | GPU | write | net parts (MB, t+q) |")
    print("|---|---|---|---|---|---|---|---|---|---|---|---|")
    worst = {}
    for n, r, wall, st, side, parts in rows:
        worst[n] = max(worst.get(n, 0), wall)
        tmb = f"{int(side.group(2)) / 1e6:.0f}" if side else "all"
        bp = f"{int(side.group(6)) / 1e6:.1f}" if side else "-"
        tf = f"{int(side.group(7)) / 1e6:.2f}" if side else "-"
        pb = sum(int(v) for v in parts.values()) / 1e6 if parts else 0
        print(f"| {n} | {r} | {wall} | {tmb} | {bp} | {tf} | {st.get('read chains', 0):.3f} | "
              f"{st.get('netting', 0):.3f} | {st.get('fill list', 0):.3f} | "
              f"{st.get('GPU fill rescoring', 0):.3f} | {st.get('write nets', 0):.3f} | "
              f"{pb:.0f} |")
    print()
    print("predicted chainNet step (slowest solo rank): " +
          ", ".join(f"N={n}: {w} ms" for n, w in sorted(worst.items())))
    print()
    print("| N | rank | wall ms | pairs | blocks (M) | chains | chained s |")
    print("|---|---|---|---|---|---|---|")
    for path in sorted(glob.glob(os.path.join(d, "c4_n*_r*.err"))):
        n, r = (int(x) for x in re.findall(r"_n(\d+)_r(\d+)", path)[0])
        t = open(path).read()
        wall = int(re.search(r"wall (\d+) ms", t).group(1))
        m = re.search(r"\[rank \d+/\d+\] (\d+) pairs, (\d+) blocks, (\d+) chains: chained in ([0-9.]+) s", t)
        if m:
            print(f"| {n} | {r} | {wall} | {m.group(1)} | {int(m.group(2)) / 1e6:.2f} | {m.group(3)} | "
                  f"{m.group(4)} |")
        else:
            print(f"| {n} | {r} | {wall} | all | 50.0 | - | - |")


if __name__ == "__main__":
    main(sys.argv[1])
