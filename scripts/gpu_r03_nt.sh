#!/bin/bash
# Probe: the kernel legs of bench.py with non-temporal k_tile loads.
set -o pipefail
out=gpurun_out/${1:-r03c}
mkdir -p $out
export TMPDIR=/tmp
GAC_TILE_NT=1 timeout -k 10 ${BENCH_LIMIT:-300} python -u bench.py --steps 1 --warmup 0 \
    --kernel-steps 10 --no-c2 --no-cpu-baseline --no-pmc > $out/bench_nt.json 2> $out/bench_nt.err
brc=$?
echo "bench nt rc=$brc"
exit $brc
