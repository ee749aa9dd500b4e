#!/bin/bash
# Round 6: the comm tests (RCCL world 1, host backend with two ranks on one
# GPU) and the chainCleaner tests (C3 at chr1 scale takes the threaded net
# parse).
set -o pipefail
out=gpurun_out/${1:-r06b}
mkdir -p $out
export TMPDIR=/tmp
( while sleep 30; do date +%T >> $out/heartbeat.txt; done ) &
hb=$!
trap "kill $hb" EXIT
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 600 --timeout-method thread tests/test_gpu_comm.py \
    tests/test_gpu_configs.py tests/test_gpu_tools.py -k "comm or cleaner or c3" > $out/tests.txt 2>&1
rc=$?
tail -5 $out/tests.txt
exit $rc
