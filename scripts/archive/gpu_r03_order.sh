#!/bin/bash
# A/B of the whole-chain plan order (GAC_WHOLE_ORDER): target order (the
# default from 4096 chains) vs set order, on the C5 kernel legs, after the
# whole-chain parity tests.  Each GPU step under its own time limit.
set -o pipefail
tag=${1:-r03k}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_scoring.py -m gpu -x -v --timeout 240 \
    --timeout-method thread -k "whole or host_ranges" > $out/gpu_tests.txt 2>&1 || exit $?
for ord in target set target; do
    GAC_WHOLE_ORDER=$ord timeout -k 10 600 python -u bench.py --steps 2 --warmup 1 --no-c2 \
        --no-cpu-baseline --kernel-steps 20 ${PMC:---no-pmc} \
        > $out/bench_$ord.json 2> $out/bench_$ord.err || exit $?
    cp $out/bench_$ord.json $out/bench_${ord}_$(date +%s).json
done
