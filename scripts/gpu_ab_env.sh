#!/bin/bash
# A/B of the C5 kernel legs under two env settings, alternating on one box:
#   gpu_ab_env.sh TAG "A_ENV" "B_ENV" [ROUNDS]   e.g. "GAC_TILE_SCAN64=1" ""
# (the bench's kernel legs only: --no-c2 --no-cpu-baseline --no-pmc, one
# headline step).  Each GPU step time-limited; stops at the first failure.
set -o pipefail
tag=$1; A=$2; B=$3; rounds=${4:-2}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
for r in $(seq $rounds); do
    for v in A B; do
        if [ $v = A ]; then e=$A; else e=$B; fi
        env $e timeout -k 10 600 python -u bench.py --steps 1 --warmup 0 --no-c2 \
            --no-cpu-baseline --kernel-steps 20 --no-pmc > $out/bench_${v}_$r.json \
            2> $out/bench_${v}_$r.err || exit $?
    done
done
python - $out <<'P'
import json, sys, glob
for f in sorted(glob.glob(sys.argv[1] + "/bench_*.json")):
    for l in open(f):
        if l.startswith("{"):
            d = json.loads(l); k = d["kernel"]; s = d["scorechain"]
            print(f.split("/")[-1], "fills k_tile %.3f" % k["kernel_ms"]["tile"],
                  "frac %.3f" % d["roofline"]["frac"], "| whole k_tile %.3f" % s["kernel_ms"]["tile"],
                  "step %.3f" % s["ms_per_step"], "frac %.3f" % s["roofline_step"]["frac"])
P
