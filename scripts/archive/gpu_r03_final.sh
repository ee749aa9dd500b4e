#!/bin/bash
# Round-3 final evidence, part A: the whole -m gpu suite, then bench.py as the
# driver runs it (defaults: C5 headline, C2 leg, kernel legs with in-run PMC
# traffic, cpu baseline).  Each GPU step time-limited; stops at the first failure.
set -o pipefail
tag=${1:-r03f}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 900 --timeout-method thread \
    > $out/gpu_tests.txt 2>&1
rc=$?
echo "pytest rc=$rc" >> $out/gpu_tests.txt
tail -2 $out/gpu_tests.txt
[ $rc -ne 0 ] && exit $rc
timeout -k 10 540 python -u bench.py > $out/bench.json 2> $out/bench.err
brc=$?
echo "bench rc=$brc"
tail -3 $out/bench.err
exit $brc
