#!/bin/bash
# Round-4 closing evidence on the committed tree, part 1: the whole -m gpu
# suite and smoke().
set -o pipefail
tag=${1:-r04final2}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
(while sleep 50; do date +%T >> $out/heartbeat.txt; done) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 1000 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests \
    --durations=25 > $out/gpu_tests.txt 2>&1 || exit $?
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.txt 2>&1 || exit $?
echo ok
