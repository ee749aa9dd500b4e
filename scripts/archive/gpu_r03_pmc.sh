#!/bin/bash
# k_tile (default again) scoring parity, then PMC passes of both kernel legs
# (fills in net order; whole chains in set and target order).  Each GPU step
# time-limited; stops at the first failure.
set -o pipefail
tag=${1:-r03o}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_scoring.py -m gpu -x -v --timeout 240 \
    --timeout-method thread > $out/gpu_tests.txt 2>&1 || exit $?
tail -1 $out/gpu_tests.txt
timeout -k 10 300 python -u bench.py --gen-only > $out/gen.txt 2>&1 || exit $?
timeout -k 10 400 python -u scripts/archive/pmc_ab.py $out fills base= > $out/pmc_fills.txt 2>&1 || exit $?
timeout -k 10 600 python -u scripts/archive/pmc_ab.py $out scorechain set=GAC_WHOLE_ORDER=set \
    target=GAC_WHOLE_ORDER=target > $out/pmc_sc.txt 2>&1 || exit $?
