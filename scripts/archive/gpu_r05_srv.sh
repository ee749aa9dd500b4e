#!/bin/bash
# The small-batch server (GAC_SMALL_SERVER=1): its GPU tests, then chainCleaner
# on C3 with and without it, alternating (scripts/c3_ab.py); the C5 headline
# with the chainNet fill arrays released late or at once (scripts/c5_ab.py).
set -o pipefail
tag=${1:-r05srv}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_scoring.py -k "small_batch_server or small_batches or host_ranges" \
    > $out/tests.txt 2>&1 || exit $?
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
    tests/test_gpu_tools.py -k chaincleaner > $out/tools.txt 2>&1 || exit $?
timeout -k 10 600 python -u scripts/c3_ab.py ${REPS:-3} > $out/c3_ab.txt 2>&1 || exit $?
if [ -n "$C5AB" ]; then
    timeout -k 10 500 python -u scripts/c5_ab.py ${C5REPS:-4} $C5AB > $out/c5_ab.txt 2>&1 || exit $?
fi
echo ok
