#!/bin/bash
# Round-5 A/B: whole chains (scoreChain) with k_tile's tiles scheduled in the
# target order of their first blocks (default) vs in set order
# (GAC_WHOLE_TILES=set); kernel legs with in-run PMC traffic, alternating;
# the scoring GPU tests under the new default first.
set -o pipefail
tag=${1:-r05tiles}
reps=${2:-2}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
(while sleep 50; do date +%T >> $out/heartbeat.txt; done) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_scoring.py > $out/gpu_tests.txt 2>&1 || exit $?
for i in $(seq 1 $reps); do
  for v in target set; do
    GAC_WHOLE_TILES=$v timeout -k 10 500 python -u bench.py --steps 1 --warmup 0 \
        --kernel-steps 20 --no-c2 --no-cpu-baseline --no-c4 \
        > $out/bench_${v}_$i.json 2> $out/bench_${v}_$i.err || exit $?
  done
done
echo ok
