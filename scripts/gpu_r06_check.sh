#!/bin/bash
# Round 6: the GPU tests touching axtChain's device DP and the small-batch
# server, then the DP profile (scripts/gpu_r06_dp.sh) on the final kernel.
set -o pipefail
out=gpurun_out/${1:-r06chk}
mkdir -p $out
export TMPDIR=/tmp
( while sleep 30; do date +%T >> $out/heartbeat.txt; done ) &
hb=$!
trap "kill $hb" EXIT
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_tools.py \
    tests/test_gpu_configs.py -k "axtchain or dp or c4 or cleaner" > $out/tests.txt 2>&1 || { tail -30 $out/tests.txt; exit 1; }
tail -3 $out/tests.txt
bash scripts/gpu_r06_dp.sh ${1:-r06chk}
