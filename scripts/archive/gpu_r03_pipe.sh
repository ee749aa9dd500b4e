#!/bin/bash
# k_tile_pipe (descriptor/block LDS-DMA of the next tile overlapped with the
# plane loads) vs k_tile (GAC_TILE_PIPE=0): scoring parity tests with the
# default, then the C5 kernel legs of both, alternating.  Each GPU step
# time-limited; stops at the first failure.
set -o pipefail
tag=${1:-r03n}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_scoring.py -m gpu -x -v --timeout 240 \
    --timeout-method thread > $out/gpu_tests.txt 2>&1 || exit $?
tail -1 $out/gpu_tests.txt
for v in 1 0 1 0; do
    GAC_TILE_PIPE=$v timeout -k 10 600 python -u bench.py --steps 1 --warmup 1 --no-c2 \
        --no-cpu-baseline --kernel-steps 20 --no-pmc > $out/bench_p$v.json 2> $out/bench_p$v.err \
        || exit $?
    cp $out/bench_p$v.json $out/bench_p${v}_$(date +%s).json
done
