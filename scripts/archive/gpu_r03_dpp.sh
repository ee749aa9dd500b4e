#!/bin/bash
# k_tile with DPP wave scans: scoring parity tests, the C5 kernel legs, then
# k_tile counter passes of the whole-chain leg.  Each GPU step time-limited.
set -o pipefail
tag=${1:-r03m}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_scoring.py -m gpu -x -v --timeout 240 \
    --timeout-method thread > $out/gpu_tests.txt 2>&1 || exit $?
tail -1 $out/gpu_tests.txt
timeout -k 10 600 python -u bench.py --steps 2 --warmup 1 --no-c2 --no-cpu-baseline \
    --kernel-steps 20 --no-pmc > $out/bench.json 2> $out/bench.err || exit $?
timeout -k 10 600 python3 scripts/archive/pmc_ab.py $out scorechain ${PMC_SPECS:-default=} \
    > $out/pmc.log 2>&1 || exit $?
