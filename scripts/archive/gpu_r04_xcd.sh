#!/bin/bash
# Round-4 A/B: k_tile's tile schedule -- per-round XCD blocks (default) vs one
# contiguous eighth of the tiles per XCD (GAC_TILE_XCD=1); the scoring tests
# under the probe first, then bench kernel legs (in-run PMC traffic)
# alternating.
set -o pipefail
tag=${1:-r04xcd}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
(while sleep 50; do date +%T >> $out/heartbeat.txt; done) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
GAC_TILE_XCD=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_scoring.py > $out/gpu_tests_xcd.txt 2>&1 || exit $?
for i in 1 2; do
  for x in 0 1; do
    GAC_TILE_XCD=$x timeout -k 10 400 python -u bench.py --steps 1 --warmup 0 --kernel-steps 20 --no-c2 \
        --no-cpu-baseline --no-c4 > $out/bench_xcd${x}_$i.json 2> $out/bench_xcd${x}_$i.err || exit $?
  done
done
echo ok
