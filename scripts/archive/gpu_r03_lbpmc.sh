#!/bin/bash
# k_tile counters on the C5 fills with and without k_plan_lb's staged window
# records (GAC_PLAN_LB=0/1): traffic, L2 hits, SQ issue/wait.
set -o pipefail
tag=${1:-r03za}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u bench.py --steps 1 --warmup 0 --no-c2 --no-cpu-baseline \
    --no-kernel > $out/bench_gen.json 2> $out/bench_gen.err || exit $?
timeout -k 10 900 python -u scripts/archive/pmc_ab.py $out fills base=GAC_PLAN_LB=0 lb=GAC_PLAN_LB=1 \
    > $out/pmc_fills.txt 2>&1 || exit $?
