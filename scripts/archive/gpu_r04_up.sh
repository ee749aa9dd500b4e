#!/bin/bash
# Round-4: upload kernels after the uniform-search change: scoring GPU tests,
# then rocprofv3 --kernel-trace --stats over a short kernel-leg bench run.
set -o pipefail
tag=${1:-r04up}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
(while sleep 50; do date +%T >> $out/heartbeat.txt; done) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_scoring.py tests/test_gpu_configs.py > $out/gpu_tests.txt 2>&1 || exit $?
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$out/prof \
    -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 1 --warmup 0 --kernel-steps 10 --no-c2 \
    --no-cpu-baseline --no-pmc --no-c4 > $GRAFT_REPO_ROOT/$out/prof_bench.json \
    2> $GRAFT_REPO_ROOT/$out/prof_bench.err || exit $?
echo ok
