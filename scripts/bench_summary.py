#!/usr/bin/env python3
"""One line per bench JSON: the headline and the kernel legs' key numbers
(k_tile times, roofline fractions, in-run PMC traffic, parity verdicts).
usage: bench_summary.py FILE.json ..."""
import json
import sys


def line(path):
    txt = open(path).read().strip().splitlines()
    d = json.loads(txt[-1])
    sc = d.get("scorechain", {})
    r = sc.get("roofline", {}) or {}
    k = d.get("kernel", {}) or {}
    fr = d.get("roofline", {}) or {}
    out = [path.split("/")[-1],
           f"hl {d.get('ms_per_step', 0):.0f}ms {d.get('value', 0):.2f}Gb/s id={d.get('identical_nets_full')}"]
    if fr:
        out.append(f"fills tile {fr.get('kernel_avg_ms', 0):.3f} frac {fr.get('frac', 0):.3f} "
                   f"traf {(fr.get('traffic') or 0) / 1e9:.2f}GB call {k.get('ms_per_step', 0):.3f}")
    if r:
        out.append(f"whole tile {r.get('kernel_avg_ms', 0):.3f} frac {r.get('frac', 0):.3f} "
                   f"traf {(r.get('traffic') or 0) / 1e9:.2f}GB x{r.get('traffic_over_algo') or 0:.2f} "
                   f"step {sc.get('ms_per_step', 0):.3f}")
    e2e = d.get("scorechain_e2e", {})
    if e2e:
        out.append(f"sc_e2e {e2e.get('ms_per_step', 0):.0f}ms id={(e2e.get('parity_full') or {}).get('identical')}")
    c3 = d.get("c3", {})
    if c3:
        out.append(f"c3 {c3.get('ms_per_step', 0):.0f}ms x{c3.get('speedup_vs_reference') or 0:.1f} "
                   f"id={c3.get('identical')}" + (f" err={c3['error'][:80]}" if "error" in c3 else ""))
    c4 = d.get("c4", {})
    if c4:
        out.append(f"c4 {c4.get('ms_per_step', 0) / 1e3:.2f}s id={(c4.get('parity_full') or {}).get('identical')}")
    return " | ".join(out)


if __name__ == "__main__":
    for p in sys.argv[1:]:
        try:
            print(line(p))
        except (OSError, ValueError, IndexError) as ex:
            print(p, "unreadable:", ex)
