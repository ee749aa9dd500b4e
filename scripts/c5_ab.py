#!/usr/bin/env python3
"""A/B of the headline tool (bin/chainNet -rescore on C5, bench.py's files)
under environment variants, alternating, outputs checked against the
reference's sha256 (tests/golden/fullscale/c5.json) after each variant's last
run; then one GAC_TIMING run per variant for its stage laps and marks.
usage: c5_ab.py REPS tag:ENV=v,ENV2=v ..."""
import os
import resource
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    reps = int(sys.argv[1])
    specs = sys.argv[2:]
    variants = []
    for sp in specs:  # tag:ENV=v,...  (@TOOL=path: another build's bin/chainNet)
        tag, _, kv = sp.partition(":")
        env = dict(os.environ)
        tool = None
        for x in filter(None, kv.split(",")):
            k, _, v = x.partition("=")
            if k == "@TOOL":
                tool = v
            else:
                env[k] = v
        variants.append((tag, env, tool))
    sys.argv = [sys.argv[0]]
    args = bench.parse()
    d, info = bench.c5_files(args)
    out = os.path.join(d, "ab")
    outs = [out + ".t.net", out + ".q.net"]
    base = bench.tool_cmd(d, out, 1, 0)
    cmd_of = lambda tool: [tool] + base[1:] if tool else base
    bench.run_tool(base, outs)  # warm the page cache
    times = {t: [] for t, _, _ in variants}
    for rep in range(reps):
        for tag, env, tool in variants:
            cmd = cmd_of(tool)
            for o in outs:
                if os.path.exists(o):
                    os.remove(o)
            ru0 = resource.getrusage(resource.RUSAGE_CHILDREN)
            t0 = time.perf_counter()
            bench.run_tool(cmd, [], env=env)
            times[tag].append((time.perf_counter() - t0) * 1e3)
            ru1 = resource.getrusage(resource.RUSAGE_CHILDREN)
            print(f"{tag} rep {rep}: {times[tag][-1]:.0f} ms (user {ru1.ru_utime - ru0.ru_utime:.2f} s, "
                  f"sys {ru1.ru_stime - ru0.ru_stime:.2f} s, minor faults "
                  f"{ru1.ru_minflt - ru0.ru_minflt})", flush=True)
    for tag, env, tool in variants:
        r = bench.run_tool(cmd_of(tool) + ["-verbose=2"], outs, env=dict(env, GAC_TIMING="1"))
        par = bench.full_parity("c5", {"in_chain_sha256": os.path.join(d, "in.chain"),
                                       "chainnet_rescore.t_net_sha256": outs[0],
                                       "chainnet_rescore.q_net_sha256": outs[1]})
        ts = sorted(times[tag])
        print(f"== {tag}: median {ts[len(ts) // 2]:.0f} ms, min {ts[0]:.0f}, all "
              f"{' '.join(f'{x:.0f}' for x in times[tag])}; nets identical {par['identical']}",
              flush=True)
        for line in r.stderr.splitlines():
            if line.startswith(("[stage]", "[mark]", "[gac_net_build]")):
                print("   " + line, flush=True)


if __name__ == "__main__":
    main()
