#!/bin/bash
# Round-3 tool probes: axtChain at C4 = 5e7 PSL blocks (ours only; the
# reference took 398 s in r02o) and C3 chainCleaner (ours + reference).
set -o pipefail
tag=${1:-r03h}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
(while sleep 50; do date +%T >> $out/heartbeat.txt; done) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 400 python -u scripts/bench_tools.py axtchain --blocks 50000000 --seed 7 --no-ref \
    > $out/c4.json 2> $out/c4.err || exit $?
timeout -k 10 400 python -u scripts/archive/c3_probe.py $out/c3.txt > $out/c3.log 2>&1 || exit $?
echo "tools ok"
