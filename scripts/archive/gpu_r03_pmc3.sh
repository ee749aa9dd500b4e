#!/bin/bash
# Memory-pipeline counters (PMC_SET=mem) of k_tile on both C5 legs.
set -o pipefail
tag=${1:-r03s}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u bench.py --steps 1 --warmup 0 --no-c2 --no-cpu-baseline \
    --no-kernel > $out/bench_gen.json 2> $out/bench_gen.err || exit $?
PMC_SET=mem timeout -k 10 600 python -u scripts/archive/pmc_ab.py $out fills base= > $out/pmc_fills.txt 2>&1 || exit $?
PMC_SET=mem timeout -k 10 600 python -u scripts/archive/pmc_ab.py $out scorechain base= > $out/pmc_sc.txt 2>&1 || exit $?
