"""Write profiles/k_tile_traffic.json (read by bench.py for roofline.traffic)
from a PMC summary (scripts/pmc_summary.py) and the bench JSON line of the
same workload.

usage: python scripts/traffic_json.py SUMMARY.json BENCH.json > profiles/k_tile_traffic.json
"""
import json
import sys


def main(summary_path, bench_path):
    s = json.load(open(summary_path))
    b = json.loads(open(bench_path).read().strip().splitlines()[-1])
    k = [name for name in s if name.startswith("gac::k_tile") and "hbm_bytes" in s[name]]
    if not k:
        sys.exit("no k_tile entry with hbm_bytes in " + summary_path)
    d = s[k[0]]
    kern = b["kernel"]
    out = {
        "kernel": k[0],
        "hbm_bytes_per_launch": d["hbm_bytes"],
        "hbm_read_bytes_per_launch": d["hbm_read_bytes"],
        "hbm_write_bytes_per_launch": d["hbm_write_bytes"],
        "algo_bytes_per_launch": b["roofline"]["algo_bytes_per_launch"],
        "workload": "rescore" if kern["workload"].startswith("chainNet") else "scorechain",
        "chains": b["config"]["chains"],
        "seed": 42,
        "ranges": kern["ranges"],
        "blocks": kern["window_blocks"],
        "order": kern.get("order", "net"),
        "source": "rocprofv3 --kernel-trace --pmc TCC_EA0_RDREQ_{32,64,128}B_sum / "
                  "TCC_EA0_WRREQ(_64B)_sum passes (scripts/archive/gpu_counters.sh), "
                  "mean per dispatch (scripts/pmc_summary.py)",
    }
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
