#!/bin/bash
# Round-5: C4 50 M host-only vs the hybrid default (alternating), then the
# bench's C3 chainCleaner leg (headline step once, other legs off); first
# the scoring and tool GPU tests (the window-search index built lazily).
set -o pipefail
tag=${1:-r05c3c4}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu \
    tests/test_gpu_scoring.py tests/test_gpu_tools.py > $out/gpu_tests.txt 2>&1 || exit $?
REPS="1 2 3 4" VARIANTS="host:GAC_AXT_DP=host hyb:GAC_DP_X=1" timeout -k 10 700 bash scripts/archive/gpu_r05_dp4.sh $tag || exit $?
timeout -k 10 600 python -u bench.py --steps 1 --warmup 0 --no-c2 --no-c4 --no-kernel --no-scorechain \
    --no-cpu-baseline > $out/bench_c3.json 2> $out/bench_c3.err || exit $?
echo ok
