#!/bin/bash
# scoring parity (test_gpu_scoring), then the bench's kernel legs (C5 fills
# + whole chains, in-run PMC traffic), no C2 / cpu-baseline legs.  Each GPU
# step time-limited; stops at the first failure.  Extra args go to bench.py.
set -o pipefail
tag=${1:-r03x}
shift
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_scoring.py -m gpu -x -v --timeout 240 \
    --timeout-method thread > $out/gpu_tests.txt 2>&1 || exit $?
tail -1 $out/gpu_tests.txt
timeout -k 10 900 python -u bench.py --steps 1 --warmup 1 --no-c2 --no-cpu-baseline \
    --kernel-steps 20 "$@" > $out/bench.json 2> $out/bench.err || exit $?
