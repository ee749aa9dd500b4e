#!/bin/bash
# The small-batch server's tests, then the per-call latency of small batches
# with and without it (scripts/archive/small_latency.py).
set -o pipefail
out=gpurun_out/${1:-r05lat}
mkdir -p $out
timeout -k 10 90 python -u -m pytest -x -v --timeout 60 --timeout-method thread -m gpu \
    tests/test_gpu_scoring.py -k "small_batch_server" > $out/tests.txt 2>&1 || exit $?
for v in ${VARIANTS:-"GAC_SMALL_SERVER=0" "GAC_SMALL_SERVER=1 GAC_SRV_TRACE=1"}; do
    echo "== $v" >> $out/lat.txt
    env $v GAC_TIMING=1 timeout -k 10 60 python -u scripts/archive/small_latency.py 2000 ${NR:-20} \
        >> $out/lat.txt 2>&1 || exit $?
done
echo ok
