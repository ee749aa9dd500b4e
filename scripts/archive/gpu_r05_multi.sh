#!/bin/bash
# Round-5 probe bundle: hybrid DP variants on C4 (gpu_r05_dp4.sh), the
# per-rank solo tables (gpu_r05_ranks.sh), the C3 leg's stage laps; first
# the scoring GPU tests (genome relayout by 16-byte accesses).
set -o pipefail
tag=${1:-r05multi}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_scoring.py > $out/gpu_tests.txt 2>&1 || exit $?
REPS="1 2 3" VARIANTS="host:GAC_AXT_DP=host hx2:GAC_DP_POOL=5 h5k:GAC_DP_POOL=5,GAC_DP_GPU_MAX=5000" \
    timeout -k 10 500 bash scripts/archive/gpu_r05_dp4.sh $tag || exit $?
timeout -k 10 500 bash scripts/gpu_r05_ranks.sh $tag || exit $?
timeout -k 10 400 python -u bench.py --steps 1 --warmup 0 --no-c2 --no-c4 --no-kernel --no-scorechain \
    --no-cpu-baseline --c3-steps 1 > $out/bench_c3.json 2> $out/bench_c3.err || exit $?
echo ok
