#!/bin/bash
# A/B of the C5 kernel legs under env settings, alternating on one box:
#   gpu_ab_env.sh TAG ROUNDS NAME=ENV[,ENV...] ...
#   e.g. gpu_ab_env.sh r03q 2 old=GAC_TILE_SCAN64=1,GAC_TILE_BLK16=1 new=
# The scoring parity tests run first; then per round every setting runs the
# bench's kernel legs (--no-c2 --no-cpu-baseline --no-pmc, one headline
# step).  Each GPU step time-limited; stops at the first failure.
set -o pipefail
tag=$1; rounds=$2; shift 2
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -s ABRT -k 10 300 python -X faulthandler -u -m pytest tests/test_gpu_scoring.py -m gpu -x -v --timeout 240 \
    --timeout-method thread > $out/gpu_tests.txt 2>&1 || exit $?
tail -1 $out/gpu_tests.txt
for r in $(seq $rounds); do
    for spec in "$@"; do
        name=${spec%%=*}; envs=${spec#*=}
        timeout -k 10 600 env ${envs//,/ } python -u bench.py --steps 1 --warmup 0 --no-c2 \
            --no-cpu-baseline --kernel-steps 20 --no-pmc > $out/bench_${name}_$r.json \
            2> $out/bench_${name}_$r.err || exit $?
    done
done
python - $out <<'P'
import json, sys, glob
for f in sorted(glob.glob(sys.argv[1] + "/bench_*.json")):
    for l in open(f):
        if l.startswith("{"):
            d = json.loads(l); k = d["kernel"]; s = d["scorechain"]
            print(f.split("/")[-1], "fills call %.3f plan %.3f k_tile %.3f" % (
                      k["ms_per_step"], k["kernel_ms"]["plan+tilemap"], k["kernel_ms"]["tile"]),
                  "frac %.3f" % d["roofline"]["frac"], "| whole k_tile %.3f" % s["kernel_ms"]["tile"],
                  "step %.3f" % s["ms_per_step"], "frac %.3f" % s["roofline_step"]["frac"])
P
