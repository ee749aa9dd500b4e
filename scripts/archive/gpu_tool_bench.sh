#!/bin/bash
# End-to-end tool timings vs the reference binaries on the GPU box's host
# (scripts/bench_tools.py); JSON lines to gpurun_out/tool_bench.jsonl.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/tool_bench.jsonl
: > $OUT
# heartbeat: long reference runs print nothing for minutes
( while true; do date +%T > gpurun_out/heartbeat; sleep 50; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
for t in "$@"; do
  echo "== $t $(date +%T)" >&2
  timeout -k 10 1500 python scripts/bench_tools.py $t >> $OUT 2>> gpurun_out/tool_bench.log; rc=$?
  echo "rc=$rc" >&2
  [ $rc -ne 0 ] && [ $rc -ge 124 ] && exit $rc
done
exit 0
