#!/bin/bash
# Round-5 A/B: the whole-chain k_tile leg (scoreChain) under chain order x
# tile schedule: set (score) order vs target order (GAC_WHOLE_ORDER=target),
# per-round XCD blocks vs one contiguous eighth of the tiles per XCD
# (GAC_TILE_XCD=1).  bench kernel legs only (the headline step once), in-run
# PMC traffic; the scoreChain e2e leg's full-scale sha checks each order.
# First the scoring / chainNet GPU tests of the tree (window scoring).
set -o pipefail
tag=${1:-r05whole}
reps=${2:-1}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
(while sleep 50; do date +%T >> $out/heartbeat.txt; done) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_scoring.py tests/test_gpu_tools.py > $out/gpu_tests.txt 2>&1 || exit $?
for i in $(seq 1 $reps); do
  for v in set:0 target:1 target:0; do
    o=${v%:*}; x=${v#*:}
    GAC_WHOLE_ORDER=$o GAC_TILE_XCD=$x timeout -k 10 500 python -u bench.py --steps 1 --warmup 0 \
        --kernel-steps 20 --no-c2 --no-cpu-baseline --no-c4 \
        > $out/bench_${o}_x${x}_$i.json 2> $out/bench_${o}_x${x}_$i.err || exit $?
  done
done
echo ok
