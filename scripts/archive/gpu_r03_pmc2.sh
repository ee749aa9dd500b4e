#!/bin/bash
# Counter inventory of the box (rocprofv3 -L) and memory-pipeline counter
# passes of k_tile on both C5 legs (fills.bin from one bench step first).
set -o pipefail
tag=${1:-r03r}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
cd /tmp && timeout -k 10 120 rocprofv3 -L > $GRAFT_REPO_ROOT/$out/counters.txt 2>&1; cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u bench.py --steps 1 --warmup 0 --no-c2 --no-cpu-baseline \
    --no-kernel > $out/bench_gen.json 2> $out/bench_gen.err || exit $?
timeout -k 10 600 python -u scripts/archive/pmc_ab.py $out fills base= > $out/pmc_fills.txt 2>&1 || exit $?
